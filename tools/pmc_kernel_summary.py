"""Table of tools/pmc_kernel.sh output: per kernel and library variant, the SQ
counters per dispatch (last dispatch of each kernel) and the derived issue /
stall fractions, VALU per wave, LDS bank conflicts per LDS cycle.
usage: python tools/pmc_kernel_summary.py gpurun_out/pmck_<tag>"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    return re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "")).replace("void ", "").strip()


def main():
    d = sys.argv[1]
    vals = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, "*_p*", "pmc_counter_collection.csv"))):
        var = os.path.basename(os.path.dirname(f)).rsplit("_p", 1)[0]
        last = {}
        rows = list(csv.DictReader(open(f)))
        for r in rows:
            k = short(r["Kernel_Name"])
            last[k] = max(last.get(k, 0), int(r["Dispatch_Id"]))
        for r in rows:
            k = short(r["Kernel_Name"])
            if int(r["Dispatch_Id"]) != last[k]:
                continue
            vals[(k, var)][r["Counter_Name"]] = vals[(k, var)].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    print("| kernel | lib | waves | VALU/wave | SALU/wave | LDS/wave | VMEM rd/wave | VMEM wr/wave | issue % | stall % | LDS conflict % |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for (k, var), c in sorted(vals.items()):
        w = c.get("SQ_WAVES", 0) or 1
        cyc = c.get("SQ_WAVE_CYCLES", 0) or 1
        lds_act = c.get("SQ_ACTIVE_INST_LDS", 0) or 1
        print("| %s | %s | %d | %.0f | %.0f | %.0f | %.0f | %.0f | %.1f | %.1f | %.1f |" % (
            k, var, w, c.get("SQ_INSTS_VALU", 0) / w, c.get("SQ_INSTS_SALU", 0) / w, c.get("SQ_INSTS_LDS", 0) / w,
            c.get("SQ_INSTS_VMEM_RD", 0) / w, c.get("SQ_INSTS_VMEM_WR", 0) / w,
            100 * c.get("SQ_ACTIVE_INST_ANY", 0) / cyc, 100 * c.get("SQ_WAIT_ANY", 0) / cyc,
            100 * c.get("SQ_LDS_BANK_CONFLICT", 0) / lds_act))


if __name__ == "__main__":
    main()
