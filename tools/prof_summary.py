"""Condense rocprofv3 CSVs (kernel stats + PMC passes) into a short markdown
table for profiles/.  usage: python tools/prof_summary.py gpurun_out/prof_<tag> > profiles/<tag>.md"""
import csv
import os
import re
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if "rocprim" in n:
        for k in ("onesweep_iteration", "onesweep_global_offsets", "partition", "scan_impl", "init_lookback",
                  "transform"):
            if k in n:
                return "rocprim::" + k
        return "rocprim::other"
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0]


def main(d):
    out = []
    ks = os.path.join(d, "trace", "trace_kernel_stats.csv")
    if os.path.exists(ks):
        agg = {}
        for r in csv.DictReader(open(ks)):
            s = short(r["Name"])
            a = agg.setdefault(s, [0, 0.0])
            a[0] += int(r["Calls"])
            a[1] += float(r["TotalDurationNs"])
        tot = sum(v[1] for v in agg.values())
        out.append("| kernel | calls | avg ms | total ms | % |\n|---|---|---|---|---|")
        for s, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            out.append("| %s | %d | %.3f | %.2f | %.1f |" % (s, c, t / c / 1e6, t / 1e6, 100 * t / tot))
    for p in sorted(os.listdir(d)):
        f = os.path.join(d, p, "pmc_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = {}
        for r in csv.DictReader(open(f)):
            k = (short(r["Kernel_Name"]), r["Counter_Name"])
            agg.setdefault(k, []).append(float(r["Counter_Value"]))
        out.append("\n%s (per dispatch, mean over %s)\n\n| kernel | counter | value |\n|---|---|---|" % (p, "dispatches"))
        for (kn, cn), v in sorted(agg.items()):
            out.append("| %s | %s | %.4g |" % (kn, cn, sum(v) / len(v)))
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1])
