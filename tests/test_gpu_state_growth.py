"""State growth over a long run.  The reference keeps a
state for every (ip, rule name) it has seen, forever (rate_limit.go:45-67); the
engine's HBM tables grow by rehashing on the device.  A rolling stream of
batches whose IPs are all new drives the IP and state tables through several
growths; size-independent checks: Len() equals the IPs seen, every sampled IP
has exactly the state its single line gave it, and the occupancy stats stay
within the 3/4 load factor."""
import pytest

import workloads as W
from banjax_amd import Config, Engine, MockBanner, RegexRateLimiter

pytestmark = pytest.mark.gpu
S = 1_000_000_000


@pytest.mark.parametrize("slot_cache", [1, 0])
def test_rolling_distinct_ips_grow_tables(slot_cache):
    eng = Engine()
    eng.debug_set_slot_cache(slot_cache)
    try:
        w = W.replace(W.CFG5, n_lines=9_000_000, n_ips=9_000_000, ipv6_pct=0)
        lim = RegexRateLimiter(Config.from_yaml(w.rules_yaml), engine=eng, banner=MockBanner())
        per = 1_500_000
        seen = 0
        samples = []
        grow = []
        for b in range(6):
            data = w.host_lines(b * per, per)
            _, out = lim.consume_lines(data, w.now_ns(b * per, per), want_results=False)
            assert out.n_lines == per
            seen += per
            st = eng.state_stats()
            grow.append(st)
            assert eng.state_len() == seen == st["ips"]
            assert st["ips"] * 4 <= st["ip_slots"] * 3 and st["states"] * 4 <= st["state_slots"] * 3
            lines = data.split(b"\n")
            for k in (0, 777, per // 2, per - 1):
                f = lines[k].split(b" ")
                samples.append((f[1].decode(), int(round(float(f[0]) * 1e9)) // 1000 * 1000))
        assert grow[-1]["rehashes"] >= 2 and grow[-1]["ip_slots"] > grow[0]["ip_slots"]
        for ip, ts in samples:
            hits, start = eng.state_get(ip, "flood10")
            assert hits == 1 and abs(start - ts) < 1000, (ip, hits, start, ts)
    finally:
        eng.close()
