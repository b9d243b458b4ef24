"""profiles/pmc_traffic.json from the FETCH_SIZE / WRITE_SIZE passes of
tools/pmc_session.sh (passes 3 and 4): HBM GB per launch of each dominant
kernel, from its last dispatch (the steady-state step).

    python tools/pmc_traffic.py gpurun_out/pmc_<tag> <source note> > profiles/pmc_traffic.json

GB = (2 x FETCH_SIZE + WRITE_SIZE) KB x 1024 / 1e9: gfx950 reports half of a
wide streaming read in FETCH_SIZE (MI355X_MICROARCH.md "HBM")."""
import csv
import glob
import json
import os
import sys

KERNELS = {"k_scan": ("k_scan<",), "k_lines": ("k_lines2<", "k_lines<"), "dfa_jobs": ("k_dfa(",)}


def last_value(d, counter, prefix):
    best = None
    for f in glob.glob(os.path.join(d, "p*", "pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or prefix not in r["Kernel_Name"]:
                continue
            did = int(r["Dispatch_Id"])
            if best is None or did > best[0]:
                best = (did, float(r["Counter_Value"]))
    return None if best is None else best[1]


def main():
    d, note = sys.argv[1], " ".join(sys.argv[2:])
    out = {"config": "cfg3 (bench.py defaults)", "source": note,
           "formula": "2 x FETCH_SIZE + WRITE_SIZE (KB; gfx950 reports half of a wide streaming read, "
                      "MI355X_MICROARCH.md HBM), last dispatch of the run", "kernels": {}}
    for k, prefixes in KERNELS.items():
        for prefix in prefixes:  # the first kernel of the list that ran (k_lines2, else k_lines)
            fe, wr = last_value(d, "FETCH_SIZE", prefix), last_value(d, "WRITE_SIZE", prefix)
            if fe is not None and wr is not None:
                break
        if fe is None or wr is None:
            continue
        out["kernels"][k] = {"kernel": prefix.rstrip("(<"), "fetch_kb_per_launch": fe, "write_kb_per_launch": wr,
                             "hbm_gb_per_launch": round((2 * fe + wr) * 1024 / 1e9, 3)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
