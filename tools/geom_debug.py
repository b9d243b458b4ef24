"""Locate the first parity difference of the tile-geometry corpus (GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_parity import GEOM_CFG, geom_lines, S  # noqa: E402
from tests.parity import Pair  # noqa: E402

t = 1700000000
for seed in [int(x) for x in (sys.argv[1:] or ["2"])]:
    data0 = geom_lines(t, seed)
    for shift in (0, seed * 7):
        pair = Pair(GEOM_CFG)
        data = b"\n" * shift + data0
        oflags, ores, _ = pair.ost.consume(pair.ocfg, data, t * S, cap=(data.count(b"\n") + 1) * 12)
        out = pair.engine.process(pair.lim.ruleset, data, t * S, copy_results=True)
        g = [(r.line_idx, r.rule_idx) for r in out.results]
        o = [(r.line_idx, r.rule_id) for r in ores]
        starts = [0]
        for i, b in enumerate(data):
            if b == 10:
                starts.append(i + 1)
        sg, so = set(g), set(o)
        print("seed", seed, "shift", shift, "gpu", len(g), "oracle", len(o), "stats", pair.engine.scan_stats(), flush=True)
        for (ln, r) in sorted(so - sg)[:5] + sorted(sg - so)[:5]:
            s0 = starts[ln]
            line = data[s0:starts[ln + 1] - 1]
            names = [x.rule for x in pair.cfg.all_rules()]
            print(" %s line %d rule %d (%s) off %d tile_off %d len %d flags g=%d o=%d" % (
                "MISSING" if (ln, r) in so else "EXTRA", ln, r, names[r], s0, s0 % 4096, len(line),
                out.line_flags[ln], oflags[ln]), flush=True)
            print("   ", line[:200], "..." if len(line) > 200 else "", flush=True)
            print("    gpu rules:", sorted(x[1] for x in g if x[0] == ln), "oracle:", sorted(x[1] for x in o if x[0] == ln))
