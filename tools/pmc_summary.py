"""Per-kernel table of the PMC passes written by tools/pmc_session.sh.

    python tools/pmc_summary.py gpurun_out/pmc_<tag> [--md]

Counters are averaged per dispatch over the last third of each kernel's
dispatches (pmc_session.sh runs 3 steps: the last one is the steady state;
--all averages every dispatch).  Derived:
  stall% = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  issue% = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  occ    = SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / CUs (average resident waves per CU;
           both counters in quad-cycles, SQ_BUSY_CYCLES summed over the SEs)
  HBM GB = (2 * FETCH_SIZE + WRITE_SIZE) KB per dispatch (gfx950 halves FETCH_SIZE
           of wide streaming reads: MI355X_MICROARCH.md "HBM")
  L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS)
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    return name.replace("void ", "").strip()


def main():
    d = sys.argv[1]
    md = "--md" in sys.argv
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    # steady state: each kernel's dispatches of the last bench step only (the
    # first step of a fresh engine creates every IP / state and is not typical)
    for f in sorted(glob.glob(os.path.join(d, "p*", "pmc_counter_collection.csv"))):
        rs = list(csv.DictReader(open(f)))
        last = {}
        for r in rs:
            last[short(r["Kernel_Name"])] = max(last.get(short(r["Kernel_Name"]), 0), int(r["Dispatch_Id"]))
        seen = collections.defaultdict(set)
        for r in rs:
            k = short(r["Kernel_Name"])
            seen[k].add(int(r["Dispatch_Id"]))
        for r in rs:
            k = short(r["Kernel_Name"])
            ids = sorted(seen[k])
            # dispatches of this kernel per step = ids / steps; keep the last step's share
            keep = ids[-max(1, len(ids) // 3):] if "--all" not in sys.argv else ids
            if int(r["Dispatch_Id"]) not in keep:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            vals[k]["_vgpr"] = [float(r["VGPR_Count"])]
    rows = []
    for k, c in vals.items():
        m = {n: sum(v) / len(v) for n, v in c.items() if v}
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        row = {
            "kernel": k,
            "vgpr": int(m.get("_vgpr", 0)),
            "waves": int(m.get("SQ_WAVES", 0)),
            "stall%": 100.0 * m.get("SQ_WAIT_ANY", 0) / wc if wc else None,
            "inst_wait%": 100.0 * m.get("SQ_WAIT_INST_ANY", 0) / wc if wc else None,
            "issue%": 100.0 * m.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else None,
            "valu/wave": m.get("SQ_INSTS_VALU", 0) / max(1, m.get("SQ_WAVES", 1)),
            "vmem_rd/wave": m.get("SQ_INSTS_VMEM_RD", 0) / max(1, m.get("SQ_WAVES", 1)),
            "lds/wave": m.get("SQ_INSTS_LDS", 0) / max(1, m.get("SQ_WAVES", 1)),
            "lds_conf%": 100.0 * m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_ACTIVE_INST_LDS"]
            if m.get("SQ_ACTIVE_INST_LDS") else None,
            "hbm_GB": (2 * m.get("FETCH_SIZE", 0) + m.get("WRITE_SIZE", 0)) * 1024 / 1e9
            if "FETCH_SIZE" in m and "WRITE_SIZE" in m else None,
            "fetch_GB": 2 * m["FETCH_SIZE"] * 1024 / 1e9 if "FETCH_SIZE" in m else None,
            "write_GB": m["WRITE_SIZE"] * 1024 / 1e9 if "WRITE_SIZE" in m else None,
            "L2hit%": 100.0 * m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
            if m.get("TCC_HIT_sum") is not None and (m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0)) else None,
        }
        rows.append(row)
    rows.sort(key=lambda r: -(r["hbm_GB"] or 0))
    cols = list(rows[0].keys()) if rows else []

    def fmt(v):
        if v is None:
            return "-"
        if isinstance(v, float):
            return "%.3f" % v if abs(v) < 10 else "%.1f" % v
        return str(v)
    if md:
        print("| " + " | ".join(cols) + " |")
        print("|" + "---|" * len(cols))
        for r in rows:
            print("| " + " | ".join(fmt(r[c]) for c in cols) + " |")
    else:
        print(" ".join("%14s" % c for c in cols))
        for r in rows:
            print(" ".join("%14s" % fmt(r[c])[:14] for c in cols))


if __name__ == "__main__":
    main()
