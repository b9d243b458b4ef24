"""Per-step kernel summary of a rocprofv3 kernel trace: for each step (from one
dispatch of `marker` to the next), the wall span, the summed kernel time, the
top kernels and the largest idle gaps between dispatches (host work, syncs,
copies the kernel trace does not show).
usage: python tools/trace_steps.py <kernel_trace.csv> [marker] [top]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    if "rocprim" in name:
        return "rocprim " + ("onesweep" if "onesweep" in name else "scan" if "scan" in name else "other")
    n = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    return re.sub(r"\s+", " ", n.split("(")[0]).strip()


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_nl_count_wt"
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == marker]
    print("%d dispatches, %d steps (marker %s)" % (len(rows), len(starts), marker))
    for si, a in enumerate(starts):
        b = starts[si + 1] if si + 1 < len(starts) else len(rows)
        step = rows[a:b]
        per, cnt = defaultdict(float), defaultdict(int)
        for r in step:
            k = short(r["Kernel_Name"])
            per[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            cnt[k] += 1
        span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e6
        print("step %d: span %.2f ms, kernels %.2f ms, %d dispatches" % (si, span, sum(per.values()), len(step)))
        for k, v in sorted(per.items(), key=lambda x: -x[1])[:top]:
            print("   %-34s %9.3f ms  x%d" % (k, v, cnt[k]))
        gaps = []
        for x, y in zip(step, step[1:]):
            g = (int(y["Start_Timestamp"]) - int(x["End_Timestamp"])) / 1e6
            gaps.append((g, short(x["Kernel_Name"]), short(y["Kernel_Name"])))
        print("   idle between dispatches: %.3f ms in all" % sum(max(0.0, g[0]) for g in gaps))
        for g in sorted(gaps, reverse=True)[:6]:
            print("   gap %.3f ms after %s, before %s" % g)


if __name__ == "__main__":
    main()
