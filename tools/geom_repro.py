"""Repeat the tile-geometry parity case (seed 2 by default) on one engine and
report every rate-limit outcome that differs from the oracle, with the state
of the (ip, rule) it belongs to (debugging the intermittent outcome mismatch).

usage: python tools/geom_repro.py [reps] [seed]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from banjax_amd import Engine  # noqa: E402
from tests.test_gpu_parity import GEOM_CFG, geom_lines, S  # noqa: E402
from tests.parity import Pair  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 2
t = 1700000000
eng = Engine()
data0 = geom_lines(t, seed)
bad = 0
for rep in range(reps):
    pair = Pair(GEOM_CFG, eng)
    for fi, data in enumerate((data0, b"\n" * (seed * 7) + data0)):
        oflags, ores, _ = pair.ost.consume(pair.ocfg, data, t * S, cap=(data.count(b"\n") + 1) * 12)
        results, out = pair.lim.consume_lines(data, t * S, want_results=True)
        lines = data.split(b"\n")
        names = [x.rule for x in pair.cfg.all_rules()]
        for k, (g, o) in enumerate(zip(out.results, ores)):
            gt = (g.line_idx, g.rule_idx, g.match_type, g.exceeded, g.seen_ip)
            ot = (o.line_idx, o.rule_id, o.match_type, o.exceeded, o.seen_ip)
            if gt != ot:
                bad += 1
                ln = g.line_idx
                ip = lines[ln].split(b" ")[1].decode()
                same = [(r.line_idx, r.match_type) for r in out.results[:k + 1] if r.rule_idx == g.rule_idx and
                        lines[r.line_idx].split(b" ")[1].decode() == ip]
                print("rep %d feed %d result %d: gpu=%s oracle=%s ip=%s rule=%s earlier same-key gpu=%s" %
                      (rep, fi, k, gt, ot, ip, names[g.rule_idx], same[-6:]), flush=True)
                print("   gpu state:", eng.state_get(ip, names[g.rule_idx]), "oracle:", pair.ost.get(ip, names[g.rule_idx]),
                      "long runs:", eng.scan_stats().get("long_runs"), flush=True)
                break
print("reps", reps, "mismatching batches", bad, flush=True)
