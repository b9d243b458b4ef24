"""Per-kernel time of one steady-state bench step from a rocprofv3 kernel trace.

    python tools/step_kernels.py gpurun_out/trace_cfg3/tr_kernel_trace.csv [marker]

A step runs from one dispatch of `marker` (default k_nl_count_wt, the first kernel
of every step) to the next; the step reported is the one before the last (the last
timed step can be followed by the bench's post-step work).
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    if "rocprim" in name:
        if "radix_sort_onesweep" in name:
            return "rocprim radix sort (onesweep)"
        if "scan" in name:
            return "rocprim scan"
        return "rocprim (other)"
    n = re.sub(r"^void ", "", name)
    n = n.replace("(anonymous namespace)::", "")
    return re.sub(r"\s+", " ", n.split("(")[0]).strip()


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_nl_count_wt"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == marker]
    if len(starts) < 3:
        sys.exit(f"need at least 3 dispatches of {marker}, found {len(starts)}")
    a, b = starts[-3], starts[-2]
    step = rows[a:b]
    per = defaultdict(float)
    for r in step:
        per[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e6
    print("One steady-state step of the default cfg3 bench (the step before the last timed one), from")
    print(f"{path} (tools/step_kernels.py); step span {span:.2f} ms, kernels {sum(per.values()):.2f} ms")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"  {v:7.3f} ms  {k}")


if __name__ == "__main__":
    main()
