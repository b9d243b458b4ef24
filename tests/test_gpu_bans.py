"""GPU parity of the device decision emission: the engine's
per-IP decision updates and formatted LogRegexBan lines (bjx_batch_bans)
against the oracle's per-trip Banner replay (internal/iptables.go:179-228,
273-294; internal/decision.go:404-439), bit-exact: same decision lists
(decision, expiry, domain), same ban-log lines in trip order, same last
banned IP.
"""
import pytest

import workloads as W
from banjax_amd import Config, MockBanner, RegexRateLimiter
from tests.parity import Pair
from tests.test_gpu_parity import EDGE_CFG, edge_lines

pytestmark = pytest.mark.gpu
S = 1_000_000_000


@pytest.fixture(scope="module")
def engine():
    from banjax_amd import Engine
    e = Engine()
    yield e
    e.close()


@pytest.mark.parametrize("name,n,batches", [("cfg1", 200_000, 3), ("cfg3", 100_000, 2), ("cfg5", 60_000, 3)])
def test_device_bans_match_oracle(engine, name, n, batches):
    w = W.scaled(W.ALL[name], n, n_ips=min(W.ALL[name].n_ips, n // 10))
    pair = Pair(w.rules_yaml, engine, device_bans=True)
    per = n // batches
    for b in range(batches):
        pair.feed(w.host_lines(b * per, per), w.now_ns(b * per, per))
    pair.compare_state()


ESC_SITE = r"""  "esc.com":
    - rule: "esc \"quoted\" <rule> & \u2028 name"
      regex: 'x'
      interval: 1
      hits_per_interval: 0
      decision: challenge
    - rule: "esc block"
      regex: 'BLOCK'
      interval: 1
      hits_per_interval: 0
      decision: iptables_block
"""
BAN_CFG = (EDGE_CFG.replace("per_site_regexes_with_rates:\n", "per_site_regexes_with_rates:\n" + ESC_SITE)
           .replace("expiring_decision_ttl_seconds: 7", "expiring_decision_ttl_seconds: 600\n"
                    "disable_logging:\n  h.com: true\n  other.com: false"))


def ban_lines(t):
    """Lines whose ban-log fields need every encoding/json escape and every
    TrimSpace edge (words[3] = path, words[5] up to '|' = UA)."""
    L = []
    add = L.append
    uas = [b"plain ua", b"  padded\t\t", b"quote\" back\\slash", b"<script>&amp;</script>", b"ctl\x01\x08\x0c\x1f\x7f",
           b"tab\there\rcr", b"bad \xff\xfe utf8", b"sep \xe2\x80\xa8 \xe2\x80\xa9 end", b"\xc2\xa0nbsp\xc2\xa0",
           b"\xe3\x80\x80ideo\xe3\x80\x80", b"\xc2\x85nel", b"ua | 200", b"| 404", b"trail \xc3", b"\xe2\x80\x8a",
           b"emoji \xf0\x9f\x98\x80 ok", b"enc \xef\xbf\xbd lit", b"surrogate \xed\xa0\x80"]
    for i, ua in enumerate(uas):
        ip = b"7.7.7.%d" % (i % 5)
        add(b"%d %s GET esc.com GET /p/%d\"<&> HTTP/1.1 %s x" % (t, ip, i, ua))
        add(b"%d %s GET esc.com GET /BLOCK%d HTTP/1.1 %s" % (t, ip, i, ua))
        add(b"%d %s GET h.com GET /x%d HTTP/1.1 %s" % (t, ip, i, ua))
    add(b"%d 7.7.7.9 GET esc.com GET /x" % t)           # < 6 words: no ban-log line
    add(b"%d 7.7.7.9 GET esc.com GET /x HTTP/1.1" % t)  # exactly 5 words
    add(b"%d 7.7.7.9 GET esc.com GET /x HTTP/1.1 " % t)  # 6th word empty
    add(b"%d 127.0.0.1 GET esc.com GET /BLOCK HTTP/1.1 ua" % t)
    return b"\n".join(L) + b"\n"


def test_device_bans_edge(engine):
    t = 1700000000
    pair = Pair(BAN_CFG, engine, device_bans=True)
    data = edge_lines(t)
    pair.feed(data, t * S)
    pair.feed(ban_lines(t), t * S + 5)
    pair.feed(data + ban_lines(t + 1), (t + 1) * S)
    pair.compare_state()
    assert pair.lim.banner.ban_log and pair.lim.banner.ban_log_temp


@pytest.mark.parametrize("tz", [19800, -36000, 0])
def test_device_bans_equal_host_replay(engine, tz):
    """Device emission vs the host Banner replay of the same trips (decision
    lists incl. ipset with standalone off, ban logs), with a local time zone."""
    w = W.scaled(W.CFG5, 40_000, n_ips=3_000)
    cfg = Config.from_yaml(w.rules_yaml.replace("expiring_decision_ttl_seconds: 10", "expiring_decision_ttl_seconds: 3600"))
    got = {}
    for dev in (False, True):
        engine.state_clear()
        banner = MockBanner()
        banner.standalone = False
        lim = RegexRateLimiter(cfg, engine=engine, banner=banner, device_bans=dev, tz_offset_s=tz)
        for b in range(2):
            lim.consume_lines(w.host_lines(b * 20_000, 20_000), w.now_ns(b * 20_000, 20_000), want_results=False)
        lim.consume_lines(ban_lines(1700000000 + 3600 * 24 * 200), (1700000000 + 3600 * 24 * 200) * S,
                          want_results=False)
        dl = {ip: (d.decision, d.expires_ns, d.domain, d.from_baskerville)
              for ip, d in banner.decision_lists.expiring.items()}
        got[dev] = (dl, banner.ban_log, banner.ban_log_temp, sorted(set(banner.ipset)), banner.banned_ip)
    assert got[True][0] == got[False][0]
    assert got[True][1] == got[False][1]
    assert got[True][2] == got[False][2]
    assert got[True][3] == got[False][3]
    assert got[True][4] == got[False][4]
    assert len(got[True][1]) > 100


@pytest.mark.parametrize("mask", [0xFF, 0xFFFF])
def test_device_bans_hash_collisions(engine, mask):
    """Tripped IPs forced onto a few hash values (test hook): the exact
    regrouping (k_ban_collide) keeps one record per distinct IP."""
    w = W.scaled(W.CFG5, 30_000, n_ips=2_000)
    engine.debug_set_ip_hash_mask(mask)
    try:
        pair = Pair(w.rules_yaml, engine, device_bans=True)
        for b in range(2):
            pair.feed(w.host_lines(b * 15_000, 15_000), w.now_ns(b * 15_000, 15_000))
        pair.compare_state()
    finally:
        engine.debug_set_ip_hash_mask(0)


@pytest.mark.parametrize("zone_name,t_change", [("America/New_York", 1699164000), ("America/New_York", 1710054000),
                                                ("Australia/Lord_Howe", 1696087800), ("Europe/Dublin", 1698541200)])
def test_device_bans_dst_zone(engine, zone_name, t_change):
    """LogRegexBan timestrings across a DST change of the local zone
    (logTime.Format in time.Local, iptables.go:187): the device's transition
    table lookup vs the host replay, and both vs Python's zoneinfo conversion
    (an independent implementation of the same tz database)."""
    import datetime as dt
    import json
    import zoneinfo
    from banjax_amd import Zone
    zone = Zone.named(zone_name)
    tz = zoneinfo.ZoneInfo(zone_name)
    cfg = Config.from_yaml(BAN_CFG)
    t0 = t_change - 3 * 3600
    lines = b"".join(b"%d.%03d 6.6.%d.%d GET esc.com GET /BLOCK%d HTTP/1.1 ua x\n" % (t0 + 97 * k, k % 1000, k // 200, k % 200, k)
                     for k in range(6 * 3600 // 97))
    logs = {}
    for dev in (False, True):
        engine.state_clear()
        lim = RegexRateLimiter(cfg, engine=engine, banner=MockBanner(), device_bans=dev, zone=zone)
        lim.consume_lines(lines, t0 * S, want_results=False)
        logs[dev] = lim.banner.ban_log
    assert logs[True] == logs[False] and len(logs[True]) >= 6 * 3600 // 97
    stamps = [(int(json.loads(l)["path"][6:]), json.loads(l)["timestring"]) for l in logs[True]]
    for k, s in stamps:
        assert s == dt.datetime.fromtimestamp(t0 + 97 * k, tz).strftime("%Y-%m-%dT%H:%M:%S"), (k, s)
    assert len({s[11:13] for _, s in stamps}) >= 5


def test_device_bans_records_only(engine):
    """BJX_BAN_RECORDS_ONLY: the same per-IP decision records as the full
    emission (decision.go:404-439 replay), no LogRegexBan lines."""
    from banjax_amd import Ruleset
    import numpy as np
    w = W.scaled(W.CFG3, 100_000, n_ips=10_000)
    cfg = Config.from_yaml(w.rules_yaml)
    rs = Ruleset(cfg)
    data, now = w.host_lines(), w.now_ns()
    got = []
    for ban_log in (True, False):
        engine.state_clear()
        engine.set_decision_lists(cfg.decision_entries)
        out = engine.process(rs, data, now, emit_bans=True, ban_log=ban_log)
        bb = engine.bans()
        got.append((out.n_trips, bb))
    (nt_full, full), (nt_rec, rec) = got
    assert nt_full == nt_rec == full.n_trips == rec.n_trips and nt_full > 0
    assert full.n_ips == rec.n_ips > 0
    assert np.array_equal(full.ips, rec.ips)
    assert full.ip_bytes == rec.ip_bytes and np.array_equal(full.ip_off, rec.ip_off)
    assert len(full.log) > 0 and rec.log == b""
    assert not rec.log_kind.any() and not rec.log_off.any()


def test_device_bans_records_only_first():
    """Records-only as the first emission of a fresh engine, then a larger
    batch (the IP-length scratch was sized only by the full
    emission): the records equal the oracle's Banner replay each time."""
    from banjax_amd import Engine
    e = Engine()
    try:
        w = W.scaled(W.CFG5, 60_000, n_ips=6_000)
        pair = Pair(w.rules_yaml, e, device_bans=True)
        pair.lim.device_ban_log = False
        for lo, n in ((0, 10_000), (10_000, 50_000)):
            out = pair.feed(w.host_lines(lo, n), w.now_ns(lo, n))
            assert out.n_trips > 0 and e.bans().log == b""
        pair.compare_state()  # decision lists and the host-written ban log vs the oracle replay
    finally:
        e.close()
