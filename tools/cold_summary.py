"""Kernels of the last cold batch in a tools/sessions/r05_cold.sh trace (time order,
kernels of at least 0.2 ms), and the total per kernel name over that batch.

    python tools/cold_summary.py gpurun_out/cold/cfg3
"""
import collections
import csv
import os
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(d, "tr_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_nl_count_wt" in r["Kernel_Name"]]
batch = rows[starts[-1]:]
t0 = int(batch[0]["Start_Timestamp"])
tot = collections.Counter()
for r in batch:
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0][:70]
    tot[name] += dur
    if dur >= 0.2:
        print("  t=%8.3f %8.3f ms  %s" % ((int(r["Start_Timestamp"]) - t0) / 1e6, dur, name))
print("batch span %.3f ms" % ((int(batch[-1]["End_Timestamp"]) - t0) / 1e6))
for k, v in tot.most_common(12):
    print("  %8.3f ms  %s" % (v, k))
