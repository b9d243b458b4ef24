import sys; sys.path.insert(0, '.')
import workloads as W
from banjax_amd import Engine
from tests.parity import Pair
eng = Engine()
for trial in range(2):
    w = W.scaled(W.CFG5H, 160_000, n_ips=20_000)
    pair = Pair(w.rules_yaml, eng)
    pair.feed(w.host_lines(0, 80_000), w.now_ns(0, 80_000))
    print("b0 stats", eng.scan_stats()["long_runs"], flush=True)
    for ip in ["1.0.0.0", "2.0.0.0", "3.0.0.0", "4.0.0.0"]:
        for n in ["burst2", "flood10", "instant"]:
            g, o = eng.state_get(ip, n), pair.ost.get(ip, n)
            if g != o: print("b0 MISMATCH", ip, n, g, o, flush=True)
    pair.feed(w.host_lines(80_000, 80_000), w.now_ns(80_000, 80_000))
    print("b1 stats", eng.scan_stats()["long_runs"], flush=True)
    for ip in ["1.0.0.0", "2.0.0.0", "3.0.0.0", "4.0.0.0"]:
        for n in ["burst2", "flood10", "instant"]:
            g, o = eng.state_get(ip, n), pair.ost.get(ip, n)
            if g != o: print("b1 MISMATCH", ip, n, g, o, flush=True)
