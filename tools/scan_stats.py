"""Per-phase device times and scan-pass counters for one workload (GPU).

usage: python tools/scan_stats.py [workload] [n_lines] [repeats]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import workloads as W  # noqa: E402
from banjax_amd import Config, Engine, Ruleset  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
w = W.scaled(W.ALL[name], n, n_ips=min(W.ALL[name].n_ips, n))
cfg = Config.from_yaml(w.rules_yaml)
rs = Ruleset(cfg)
e = Engine()
e.set_decision_lists(cfg.decision_entries)
t, nb = w.device_lines(0)
for i in range(reps):
    e.state_clear()
    o = e.process(rs, None, w.now_ns(), device_ptr=t.data_ptr(), nbytes=nb)
    print(json.dumps({"workload": name, "lines": o.n_lines, "bytes": nb, "results": o.n_results,
                      "events": o.n_events, "trips": o.n_trips, "device_ms": round(o.device_ms, 3),
                      "scan_ms": round(o.match_kernel_ms, 3), "scan_GBps": round(nb / o.match_kernel_ms / 1e6, 1),
                      "phases": e.phase_ms(), "kernel_ms": e.kernel_ms(), "stats": e.scan_stats()}), flush=True)
