"""Hot-key rate limiting: one IP holding a
large share of a batch makes a single (ip, rule name) run that crosses many
k_apply chunks; k_long_runs applies it with block-parallel window search and
the closed-form trip rule, or serially when limits differ or timestamps go
backwards.  Against the oracle's sequential RegexRateLimitStates.Apply
(reference internal/rate_limit.go:37-78), bit-exact."""
import pytest

import workloads as W
from banjax_amd import Engine
from tests.parity import Pair

pytestmark = pytest.mark.gpu
S = 1_000_000_000


@pytest.fixture(scope="module")
def engine():
    e = Engine()
    yield e
    e.close()


@pytest.mark.parametrize("slot_cache,sort2", [(1, "1"), (0, "1"), (1, "2")])
def test_hot_key_workload(engine, slot_cache, sort2, monkeypatch):
    """cfg5h shape (one IP sends 25% of the lines), oracle-sized, two batches;
    with the state-slot cache of k_st_claim on and off (bit-exact both ways),
    and through the two-level grouping (BJX_SORT2=2: the hot IP's buckets
    overflow and take the full sort on their own)."""
    monkeypatch.setenv("BJX_SORT2", sort2)
    w = W.scaled(W.CFG5H, 160_000, n_ips=20_000)
    engine.debug_set_slot_cache(slot_cache)
    try:
        engine.state_clear()
        pair = Pair(w.rules_yaml, engine)
        pair.feed(w.host_lines(0, 80_000), w.now_ns(0, 80_000))
        pair.feed(w.host_lines(80_000, 80_000), w.now_ns(80_000, 80_000))
        pair.compare_state(["1.0.0.0", "2.0.0.0", "3.0.0.0"])
    finally:
        engine.debug_set_slot_cache(-1)


HOT_CFG = """
regexes_with_rates:
  - rule: "shared"
    regex: 'GET'
    interval: %s
    hits_per_interval: %d
    decision: challenge
  - rule: "shared"
    regex: 'POST'
    interval: %s
    hits_per_interval: %d
    decision: nginx_block
  - rule: "every"
    regex: '.*'
    interval: 0.25
    hits_per_interval: -1
    decision: challenge
expiring_decision_ttl_seconds: 10
"""


def _hot_lines(t0_ms, n, step_ms=1, backwards_every=0, post_every=7):
    out = []
    for k in range(n):
        t = t0_ms + k * step_ms
        if backwards_every and k % backwards_every == 0:
            t -= 5000
        m = "POST" if k % post_every == 0 else "GET"
        ip = "6.6.6.6" if k % 10 else "7.7.7.%d" % (k % 200)
        out.append("%d.%03d %s %s h.com %s /x HTTP/1.1 ua" % (t // 1000, t % 1000, ip, m, m))
    return ("\n".join(out) + "\n").encode()


@pytest.mark.parametrize("iv1,lim1,iv2,lim2,back", [
    ("2", 37, "2", 37, 0),      # uniform, monotone: window search + closed form
    ("0.5", 0, "0.5", 0, 0),    # every hit trips
    ("3", -1, "3", -1, 0),      # limit < 0
    ("2", 37, "2", 5, 0),       # rules sharing the name with different limits: serial
    ("2", 37, "2", 37, 97),     # timestamps going backwards: serial
])
@pytest.mark.parametrize("slot_cache,sort2", [(1, "1"), (0, "1"), (1, "2")])
def test_hot_key_runs(engine, iv1, lim1, iv2, lim2, back, slot_cache, sort2, monkeypatch):
    monkeypatch.setenv("BJX_SORT2", sort2)
    engine.debug_set_slot_cache(slot_cache)
    try:
        engine.state_clear()
        pair = Pair(HOT_CFG % (iv1, lim1, iv2, lim2), engine)
        t0 = 1700000000_000
        pair.feed(_hot_lines(t0, 30_000, backwards_every=back), t0 * 1_000_000)
        pair.feed(_hot_lines(t0 + 30_000, 30_000, backwards_every=back), (t0 + 30_000) * 1_000_000)
        pair.compare_state(["6.6.6.6", "7.7.7.1"])
    finally:
        engine.debug_set_slot_cache(-1)


def test_hot_key_reload_lowers_limit(engine):
    """The stored window carries more hits than the reloaded rule allows (h0 >
    limit): the first hit of the continuing window trips."""
    t0 = 1700000000_000
    pair = Pair(HOT_CFG % ("100", 5000, "100", 5000), engine)
    pair.feed(_hot_lines(t0, 3_000), t0 * 1_000_000)
    from banjax_amd import Config, RegexRateLimiter  # noqa: F401
    from tests.parity import oracle_config
    new = HOT_CFG % ("100", 40, "100", 40)
    pair.cfg = Config.from_yaml(new)
    pair.ocfg = oracle_config(pair.cfg)
    pair.lim.reload(pair.cfg)
    pair.feed(_hot_lines(t0 + 3_000, 20_000), (t0 + 3_000) * 1_000_000)
    pair.compare_state(["6.6.6.6"])


def _spread_lines(t0_ms, n, n_ips=3000):
    out = []
    for k in range(n):
        t = t0_ms + k
        m = "POST" if k % 7 == 0 else "GET"
        out.append("%d.%03d 10.%d.%d.%d %s h.com %s /x HTTP/1.1 ua" % (t // 1000, t % 1000, (k % n_ips) >> 16,
                                                                   ((k % n_ips) >> 8) & 255, k % 256, m, m))
    return ("\n".join(out) + "\n").encode()


def test_two_level_hot_key_hold(engine, monkeypatch):
    """The default grouping policy (no BJX_SORT2), with its batch-size gate
    lowered (BJX_SORT2_MIN=0) and the hold shortened to 2 batches: a batch with
    more than 1/8 of its events in oversized buckets runs two-level (those
    buckets through the full sort), the next 2 batches keep the full sort
    (grouping 0), and the one after returns to two-level grouping.  BJX_CHECK=1
    verifies every sorted outcome is written exactly once on both paths
    (k_bucket_apply, and k_apply + k_big_outs for the oversized buckets).
    Bit-exact against the oracle throughout."""
    monkeypatch.delenv("BJX_SORT2", raising=False)
    monkeypatch.setenv("BJX_SORT2_MIN", "0")
    monkeypatch.setenv("BJX_SORT2_HOLD", "2")
    monkeypatch.setenv("BJX_CHECK", "1")
    engine.state_clear()
    pair = Pair(HOT_CFG % ("2", 37, "2", 37), engine)
    t0 = 1700000000_000
    out = pair.feed(_hot_lines(t0, 30_000), t0 * 1_000_000)
    g = engine.scan_stats()["grouping"]
    assert g - 1 > out.n_events // 8, (g, out.n_events)  # two-level, the hot buckets fully sorted
    seen = []
    for b in range(3):
        t = t0 + 30_000 * (b + 1)
        pair.feed(_spread_lines(t, 20_000), t * 1_000_000)
        seen.append(engine.scan_stats()["grouping"])
    assert seen[0] == 0 and seen[1] == 0 and seen[2] == 1, seen
    pair.compare_state(["6.6.6.6", "7.7.7.1", "10.0.1.1"])
