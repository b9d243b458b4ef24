"""Steady-state rate-limit tables: phases and table sizes over consecutive
batches of one workload, state kept between batches (GPU).

usage: python tools/state_probe.py [workload] [n_lines] [batches]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import workloads as W  # noqa: E402
from banjax_amd import Config, Engine, Ruleset  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 125_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
w = W.scaled(W.ALL[name], n, n_ips=min(W.ALL[name].n_ips, n))
cfg = Config.from_yaml(w.rules_yaml)
rs = Ruleset(cfg)
e = Engine(ip_arena_bytes=256 << 20)
e.set_decision_lists(cfg.decision_entries)
t, nb = w.device_lines(0)
for i in range(reps):
    o = e.process(rs, None, w.now_ns(), device_ptr=t.data_ptr(), nbytes=nb)
    print(json.dumps({"batch": i, "lines": o.n_lines, "events": o.n_events, "trips": o.n_trips,
                      "device_ms": round(o.device_ms, 3), "phases": e.phase_ms(), "stats": e.scan_stats()}), flush=True)
