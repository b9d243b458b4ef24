import sys; sys.path.insert(0, '.')
import workloads as W
from banjax_amd import Engine
from tests.parity import Pair
eng = Engine()
bad = 0
for trial in range(6):
    w = W.scaled(W.CFG5H, 160_000, n_ips=20_000)
    pair = Pair(w.rules_yaml, eng)
    for b in range(2):
        pair.feed(w.host_lines(b * 80_000, 80_000), w.now_ns(b * 80_000, 80_000))
        lr = eng.scan_stats()["long_runs"]
        for ip in ["1.0.0.0", "2.0.0.0", "3.0.0.0", "4.0.0.0", "5.0.0.0"]:
            for n in ["burst2", "flood10", "instant"]:
                g, o = eng.state_get(ip, n), pair.ost.get(ip, n)
                if g != o:
                    bad += 1
                    print("trial", trial, "batch", b, "long_runs", lr, "MISMATCH", ip, n, g, o, flush=True)
print("done bad", bad)
