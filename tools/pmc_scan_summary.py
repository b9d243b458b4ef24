"""Per-kernel PMC table for tools/sessions/r05_pmc_scan.sh output (last dispatch of each
kernel per pass: the second scan_stats batch, warm).

    python tools/pmc_scan_summary.py gpurun_out/pmc_<tag> [cfg3|cfg4 ...]
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    return re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "")).replace("void ", "").strip()


def load(d, cfg):
    vals = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, cfg + "_p*", "pmc_counter_collection.csv"))):
        rows = list(csv.DictReader(open(f)))
        last = {}
        for r in rows:
            k = short(r["Kernel_Name"])
            last[k] = max(last.get(k, -1), int(r["Dispatch_Id"]))
        for r in rows:
            k = short(r["Kernel_Name"])
            if int(r["Dispatch_Id"]) == last[k]:
                vals[k][r["Counter_Name"]] = vals[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return vals


def main():
    d = sys.argv[1]
    for cfg in sys.argv[2:] or ["cfg3", "cfg4"]:
        for k, v in sorted(load(d, cfg).items()):
            w = v.get("SQ_WAVES", 1) or 1
            wc = v.get("SQ_WAVE_CYCLES", 1) or 1
            out = {
                "valu/wave": v.get("SQ_INSTS_VALU", 0) / w,
                "salu/wave": v.get("SQ_INSTS_SALU", 0) / w,
                "lds/wave": v.get("SQ_INSTS_LDS", 0) / w,
                "vmem_rd/wave": v.get("SQ_INSTS_VMEM_RD", 0) / w,
                "vmem_wr/wave": v.get("SQ_INSTS_VMEM_WR", 0) / w,
                "stall%": 100 * v.get("SQ_WAIT_ANY", 0) / wc,
                "inst_wait%": 100 * v.get("SQ_WAIT_INST_ANY", 0) / wc,
                "lds_issue_wait%": 100 * v.get("SQ_WAIT_INST_LDS", 0) / wc,
                "issue%": 100 * v.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                "valu_active%": 100 * v.get("SQ_ACTIVE_INST_VALU", 0) / wc,
                "lds_active%": 100 * v.get("SQ_ACTIVE_INST_LDS", 0) / wc,
                "lds_conf%": 100 * v.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, v.get("SQ_ACTIVE_INST_LDS", 0)),
                "fetch_GB": v.get("FETCH_SIZE", 0) * 1024 / 1e9,
                "write_GB": v.get("WRITE_SIZE", 0) * 1024 / 1e9,
                "L2hit%": 100 * v.get("TCC_HIT_sum", 0) / max(1.0, v.get("TCC_HIT_sum", 0) + v.get("TCC_MISS_sum", 0)),
            }
            print(cfg, k, " ".join("%s=%.4g" % kv for kv in out.items()))


if __name__ == "__main__":
    main()
