"""Repeat the tile-geometry parity batch (tests/test_gpu_parity.py seed 2) on a
fresh state and report the first mismatch with the IPs and states involved.

    python tools/dbg_geom.py [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_parity import GEOM_CFG, geom_lines  # noqa: E402
from tests.parity import Pair  # noqa: E402
from banjax_amd import Engine  # noqa: E402

S = 1_000_000_000
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
e = Engine()
t = 1700000000
for seed in (2, 1, 3):
    data = geom_lines(t, seed)
    lines = data.split(b"\n")
    for rep in range(reps):
        pair = Pair(GEOM_CFG, e)
        oflags, ores, _ = pair.ost.consume(pair.ocfg, data, t * S, cap=(data.count(b"\n") + 1) * (pair.n_rules + 1))
        out = e.process(pair.lim.ruleset, data, t * S, copy_results=True)
        bad = None
        for k, (g, o) in enumerate(zip(out.results, ores)):
            gt = (g.line_idx, g.rule_idx, g.rule_pos, g.skip_host, g.seen_ip, g.match_type, g.exceeded)
            ot = (o.line_idx, o.rule_id, o.rule_pos, o.skip_host, o.seen_ip, o.match_type, o.exceeded)
            if gt != ot:
                bad = (k, gt, ot)
                break
        print("seed", seed, "rep", rep, "n_results", out.n_results, len(ores), "first mismatch", bad, flush=True)
        if bad:
            ln = lines[bad[1][0]]
            ip = ln.split(b" ")[1]
            print("  line:", ln[:80], flush=True)
            names = sorted(set(r.rule for r in pair.cfg.all_rules()))
            for nm in names:
                print("  state", ip, nm, "gpu", e.state_get(ip, nm), "oracle", pair.ost.get(ip, nm), flush=True)
            print("  gpu Len", e.state_len(), "oracle Len", len(pair.ost), flush=True)
