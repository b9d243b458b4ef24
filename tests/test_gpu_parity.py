"""GPU parity: the HIP engine (through the C ABI) against the oracle, bit-exact.

Restates the reference's hot-path tests (internal/regex_rate_limiter_test.go)
through the engine, then checks every BASELINE.json workload shape at sizes
the oracle finishes in seconds, edge-case lines, and size-independent
properties at larger sizes.
"""
import random

import pytest

import workloads as W
from banjax_amd import Config, Engine, MockBanner, RegexRateLimiter, Ruleset, consume_line
from oracle import oracle as O
from tests.parity import Pair, oracle_config

pytestmark = pytest.mark.gpu
S = 1_000_000_000


@pytest.fixture(scope="module")
def engine():
    e = Engine()
    yield e
    e.close()


TEST_CONSUME_LINE_CFG = r"""
regexes_with_rates:
  - decision: nginx_block
    rule: 'rule1'
    regex: 'GET example\.com GET .*'
    interval: 5
    hits_per_interval: 2
  - decision: challenge
    rule: 'rule2'
    regex: 'POST .*'
    interval: 5
    hits_per_interval: 1
per_site_regexes_with_rates:
  per-site.com:
    - decision: nginx_block
      hits_per_interval: 0
      interval: 1
      regex: .*blockme.*
      rule: "instant block"
"""


def test_consume_line_sequence(engine):
    """regex_rate_limiter_test.go:77-260 TestConsumeLine, through the GPU."""
    engine.state_clear()
    lim = RegexRateLimiter(Config.from_yaml(TEST_CONSUME_LINE_CFG), engine=engine, banner=MockBanner())
    t0 = 1700000000.123456
    now = int(t0 * 1e9)
    ua = "AppleWebKit/537.36 (KHTML, like Gecko) Chrome/51.0.2704.103 Safari/537.36 -"
    get = " 1.2.3.4 GET example.com GET /whatever HTTP/1.1 " + ua
    post = " 1.2.3.4 POST example.com POST /whatever HTTP/1.1 " + ua
    consume_line(lim, "%f" % t0 + get, now)
    assert lim.states.get("1.2.3.4")["rule1"][0] == 1 and lim.banner.banned_ip == ""
    consume_line(lim, "%f" % (t0 + 4) + get, now)
    assert lim.states.get("1.2.3.4")["rule1"][0] == 2 and lim.banner.banned_ip == ""
    consume_line(lim, "%f" % (t0 + 5.5) + get, now)
    assert lim.states.get("1.2.3.4")["rule1"][0] == 1 and lim.banner.banned_ip == ""
    consume_line(lim, "%f" % (t0 + 6.5) + post, now)
    st = lim.states.get("1.2.3.4")
    assert st["rule1"][0] == 1 and st["rule2"][0] == 1 and lim.banner.banned_ip == ""
    r = consume_line(lim, "%f" % (t0 + 7.0) + post, now)
    st = lim.states.get("1.2.3.4")
    assert st["rule1"][0] == 1 and st["rule2"][0] == 0 and lim.banner.banned_ip == "1.2.3.4"
    assert [x.rule_name for x in r.rule_results] == ["rule2"] and r.rule_results[0].rate_limit_result.exceeded
    consume_line(lim, "%f 1.6.6.6 GET per-site.com GET /blockme/?a HTTP/1.1 %s" % (t0 + 20, ua), now)
    assert lim.states.get("1.6.6.6") is not None
    consume_line(lim, "%f 1.6.6.7 GET no-per-site.com GET /blockme/?a HTTP/1.1 %s" % (t0 + 22, ua), now)
    assert lim.states.get("1.6.6.7") is None


def test_consume_line_hosts_to_skip(engine):
    """regex_rate_limiter_test.go:262-297 TestConsumeLineHostsToSkip."""
    engine.state_clear()
    cfg = Config.from_yaml(r"""
regexes_with_rates:
  - decision: nginx_block
    rule: 'rule1'
    regex: '^GET https?:\/\/\.*'
    interval: 5
    hits_per_interval: 2
    hosts_to_skip:
      skiphost.com: true
""")
    lim = RegexRateLimiter(cfg, engine=engine, banner=MockBanner())
    t = 1700000000.5
    consume_line(lim, "%f 1.2.3.4 GET skiphost.com GET /whatever HTTP/1.1 x" % t, int(t * 1e9))
    assert lim.states.get("1.2.3.4") is None
    r = consume_line(lim, "%f 1.2.3.4 GET skiphost.com GET http://x HTTP/1.1 x" % t, int(t * 1e9))
    assert lim.states.get("1.2.3.4") is None
    assert len(r.rule_results) == 0


def test_per_site_regex_stress(engine):
    """regex_rate_limiter_test.go:299-365 TestPerSiteRegexStress (10,000 global
    rules, every line trips its own rule), seeded."""
    rnd = random.Random(11)
    n = 10000
    doms, paths, rules = [], [], ["regexes_with_rates:"]
    for i in range(n):
        d = "%s%d.%s" % (rnd.choice(["acme", "shop", "news", "blog"]), i, rnd.choice(["com", "org", "net"]))
        p = "/%s/%d" % (rnd.choice(["a", "img", "api"]), rnd.randrange(10 ** 6))
        rules.append("  - decision: nginx_block\n    rule: 'rule%d'\n    regex: 'GET %s GET \\%s HTTP\\/[0-2.]+ .*'\n"
                     "    interval: 1\n    hits_per_interval: 0" % (i, d.replace(".", "\\."), p))
        doms.append(d)
        paths.append(p)
    pair = Pair("\n".join(rules) + "\n", engine)
    base = 1700000000
    lines, ips = [], []
    for j in range(n):
        ip = "%d.%d.%d.%d" % (rnd.randrange(1, 255), rnd.randrange(256), rnd.randrange(256), rnd.randrange(256))
        ips.append(ip)
        lines.append("%f %s GET %s GET %s HTTP/2.0 Mozilla/5.0 (X11)\n" % (float(base + j), ip, doms[j], paths[j]))
    data = "".join(lines).encode()
    out = pair.feed(data, base * S)  # reference: lines at time.Now()+j, never old
    assert out.n_trips == n
    # 10,000 global rules: no line-kernel pass, the wide per-line kernel (decide_wide) takes every line
    assert pair.engine.line_kernel()[0] == "k_parse_match"
    for j in range(0, n, 997):
        assert pair.engine.state_get(ips[j], "rule%d" % j) == (0, (base + j) * S)
    pair.compare_state(ips[:50])


@pytest.mark.parametrize("name,n_lines,batches", [
    ("cfg1", 200_000, 3), ("cfg2", 40_000, 2), ("cfg3", 100_000, 3), ("cfg4", 1_500, 2), ("cfg5", 60_000, 2)])
def test_workload_parity(engine, name, n_lines, batches):
    """Every BASELINE.json config shape, oracle-sized, split into batches so the
    HBM state carries across bjx_process_batch calls; each through k_lines2."""
    w = W.scaled(W.ALL[name], n_lines, n_ips=min(W.ALL[name].n_ips, n_lines // 3 + 1))
    pair = Pair(w.rules_yaml, engine)
    per = (n_lines + batches - 1) // batches
    ips = set()
    for b in range(batches):
        first, cnt = b * per, min(per, n_lines - b * per)
        data = w.host_lines(first, cnt)
        for ln in data.split(b"\n")[:200]:
            parts = ln.split(b" ")
            if len(parts) > 2:
                ips.add(parts[1].decode())
        pair.feed(data, w.now_ns(first, cnt))
        # every BASELINE config runs the window kernel (cfg2: 100 positions,
        # 2-word masks, literal ids past 32)
        assert pair.engine.line_kernel()[0] == "k_lines2", name
    pair.compare_state(sorted(ips)[:100])


@pytest.mark.parametrize("line_pass", [False, True])
def test_wide_scope_workload(engine, line_pass, monkeypatch):
    """cfg2k: 1,000 global rules in the TestPerSiteRegexStress shape
    (regex_rate_limiter_test.go:299-365), so every line's scope has 1,000
    positions: past k_lines2's 128-position tables, no line-kernel pass runs and
    the wide per-line kernel (k_parse_match, decide_wide) takes every line (the
    bench line of this shape is in DESIGN.md §5).  Bit-exact against the oracle
    over two batches, and again with BJX_LINES=1 (the old k_lines pass first)."""
    if line_pass:
        monkeypatch.setenv("BJX_LINES", "1")
    w = W.scaled(W.CFG2K, 12_000, n_ips=3_000)
    pair = Pair(w.rules_yaml, engine)
    for b in range(2):
        pair.feed(w.host_lines(b * 6_000, 6_000), w.now_ns(b * 6_000, 6_000))
        assert pair.engine.line_kernel()[0] == ("k_lines" if line_pass else "k_parse_match")
    pair.compare_state([ln.split(b" ")[1].decode() for ln in w.host_lines(0, 50).split(b"\n")[:50] if ln])


EDGE_CFG = r"""
global_decision_lists:
  allow:
    - 20.20.20.20
    - 2001:db8::/32
    - 10.0.0.0/8
    - not-an-ip
    - ::ffff:5.6.7.8
  challenge:
    - 8.8.8.8
per_site_decision_lists:
  "h.com":
    allow:
      - 171.171.171.0/24
      - 01.2.3.4
      - ::ffff:9.9.0.0/112
regexes_with_rates:
  - rule: "all"
    regex: '.*'
    interval: 2
    hits_per_interval: 1
    decision: challenge
  - rule: "wb"
    regex: '\bx\b'
    interval: 1
    hits_per_interval: 0
    decision: nginx_block
  - rule: "anch"
    regex: '^GET \S+ GET /$'
    interval: 10
    hits_per_interval: 0
    decision: iptables_block
  - rule: "utf"
    regex: '(?i)straße|\x{FFFD}k'
    interval: 1
    hits_per_interval: 0
    decision: nginx_block
  - rule: "neg"
    regex: '[^\x00-\x7f]'
    interval: 100
    hits_per_interval: 3
    decision: challenge
per_site_regexes_with_rates:
  "h.com":
    - rule: "all"
      regex: 'POST'
      interval: 0.5
      hits_per_interval: -1
      decision: nginx_block
expiring_decision_ttl_seconds: 7
"""


def edge_lines(t):
    L = []
    add = L.append
    add(b"")
    add(b"garbage")
    add(b"1.5 1.2.3.4")
    add(b"%d 1.2.3.4 GET" % t)
    add(b"%d 1.2.3.4 GET h.com" % t)
    add(b"%d 1.2.3.4 GET h.com GET / HTTP/1.1 ua" % t)
    add(b"%d.5 1.2.3.4 GET h.com GET / x" % (t - 11))
    add(b"%d.5 1.2.3.4 GET h.com GET / x" % (t - 9))
    for ts in [b"1e9", b"1_700_000_000.25", b"0x1.95p30", b"+1700000000", b"-5", b"inf", b"NaN", b"1e400", b"1e-400",
               b".5", b"5.", b"1700000000.123456789012345678901", b"00001700000000", b"1.2.3", b"", b"0x", b"1__0",
               b"170000000000000000000000000000", b"1700000000.000000000000000000000000001"]:
        add(ts + b" 3.3.3.3 GET h.com GET /x HTTP/1.1 ua")
    for ip in [b"20.20.20.20", b"2001:db8::7", b"10.9.8.7", b"not-an-ip", b"5.6.7.8", b"::ffff:20.20.20.20",
               b"171.171.171.5", b"01.2.3.4", b"9.9.1.1", b"9.9.0.1", b"::ffff:9.9.0.7", b"1.2.3.4%eth0", b"",
               b"256.1.1.1", b"::", b"2001:db9::1", b"8.8.8.8"]:
        add(b"%d " % t + ip + b" GET h.com GET / HTTP/1.1 ua")
        add(b"%d " % t + ip + b" POST other.com POST / HTTP/1.1 ua")
    add(b"%d 4.4.4.4 GET h.com GET x y\r" % t)
    add(b"%d 4.4.4.4 GET h.com GET / x STRASSE" % t)
    add(b"%d 4.4.4.4 GET h.com GET / x stra\xc3\x9fe" % t)
    add(b"%d 4.4.4.4 GET h.com GET / x \xffk" % t)
    add(b"%d 4.4.4.4 GET h.com GET / x \xe2\x84\xaak" % t)
    add(b"%d 4.4.4.4 GET h.com GET / x \xc3" % t)
    add(b"%d 4.4.4.4 GET h.com GET / x x" % t)
    add(b"%d 4.4.4.4 GET h.com GET / x_x" % t)
    add(b"%d 4.4.4.4  h.com GET / " % t)
    add(b"%d 4.4.4.4 GET  GET / x" % t)
    add(b"%d  GET h.com GET / x" % t)
    add(b"%d 4.4.4.4 GET h.com GET /" % t)
    return b"\n".join(L) + b"\npartial-line-without-newline"


def test_edge_lines(engine):
    t = 1700000000
    pair = Pair(EDGE_CFG, engine)
    data = edge_lines(t)
    pair.feed(data, t * S)
    pair.feed(data, (t + 1) * S)  # replay: carried state, trips, escalations
    pair.compare_state(["1.2.3.4", "3.3.3.3", "4.4.4.4", "8.8.8.8", "", "::", "not-an-ip"])


def test_regex_corpus(engine):
    """Random rules x random texts, GPU engine vs oracle regexp."""
    rnd = random.Random(5)
    atoms = [r"a", r"b", r"\d", r"\w", r"\W", r"\s", r".", r"[a-c]", r"[^ab]", r"(?i:K)", r"\b", r"\B", r"^", r"$",
             r"é", r"\x{FFFD}", r"(a|bc)", r"x?", r"y+", r"z*", r"[[:upper:]]", r"\.", r" "]
    pats = []
    for _ in range(60):
        p = "".join(rnd.choice(atoms) for _ in range(rnd.randrange(1, 5)))
        if rnd.random() < 0.3:
            p = p + "{1,3}" if not p.endswith(("?", "+", "*", "}")) else p
        if O.compile_error(p) is None:
            pats.append(p)
    yaml_rules = ["regexes_with_rates:"]
    for i, p in enumerate(pats):
        yaml_rules.append("  - rule: 'r%d'\n    regex: '%s'\n    interval: 1\n    hits_per_interval: 1000000\n"
                          "    decision: challenge" % (i, p.replace("'", "''")))
    pair = Pair("\n".join(yaml_rules) + "\n", engine)
    alpha = [b"a", b"b", b"c", b"K", b"k", b"1", b" ", b"_", b".", b"\xc3\xa9", b"\xff", b"\xe2\x84\xaa", b"-", b"x",
             b"y", b"z", b"\r"]
    lines = []
    for j in range(3000):
        body = b"".join(rnd.choice(alpha) for _ in range(rnd.randrange(0, 12)))
        lines.append(b"1700000000 9.9.9.%d GET h%d.com " % (j % 250, j % 7) + body)
    pair.feed(b"\n".join(lines) + b"\n", 1700000000 * S)


def test_batching_is_associative(engine):
    """Size-independent property at a larger size: one batch == four batches
    (same trips in the same order, same final state)."""
    w = W.scaled(W.CFG3, 2_000_000, n_ips=50_000)
    data = w.host_lines()
    now = w.now_ns()
    engine.state_clear()
    rs_cfg = Config.from_yaml(w.rules_yaml)
    lim = RegexRateLimiter(rs_cfg, engine=engine, banner=MockBanner())
    _, one = lim.consume_lines(data, now, want_results=False)
    trips_one = [(t.line_idx, t.rule_idx) for t in one.trips]
    dump_one = engine.state_dump()
    engine.state_clear()
    lim2 = RegexRateLimiter(rs_cfg, engine=engine, banner=MockBanner())
    lines = data.split(b"\n")[:-1]
    q = len(lines) // 4
    trips_four, base = [], 0
    for k in range(4):
        chunk = b"\n".join(lines[k * q:(k + 1) * q if k < 3 else len(lines)]) + b"\n"
        _, o = lim2.consume_lines(chunk, now, want_results=False)
        trips_four += [(t.line_idx + base, t.rule_idx) for t in o.trips]
        base += o.n_lines
    assert trips_one == trips_four
    assert sorted(dump_one.split("\n\n")) == sorted(engine.state_dump().split("\n\n"))


GEOM_CFG = r"""
regexes_with_rates:
  - rule: "all"
    regex: '.*'
    interval: 5
    hits_per_interval: 50
    decision: challenge
  - rule: "equiv"
    regex: 'needle'
    interval: 1
    hits_per_interval: 2
    decision: nginx_block
  - rule: "nonequiv"
    regex: 'haystack[0-9]+x'
    interval: 1
    hits_per_interval: 1
    decision: challenge
  - rule: "ci"
    regex: '(?i)foobar'
    interval: 1
    hits_per_interval: 3
    decision: challenge
  - rule: "anch"
    regex: '^GET \S+ GET /a'
    interval: 1
    hits_per_interval: 4
    decision: challenge
  - rule: "scan"
    regex: '[0-9]{3}z'
    interval: 1
    hits_per_interval: 0
    decision: nginx_block
  - rule: "alt"
    regex: 'alpha(beta|gamma)delta|omega{2,}'
    interval: 2
    hits_per_interval: 1
    decision: challenge
per_site_regexes_with_rates:
  "h.com":
    - rule: "site"
      regex: 'sitelit'
      interval: 1
      hits_per_interval: 0
      decision: nginx_block
    - rule: "equiv"
      regex: 'needle\d'
      interval: 1
      hits_per_interval: 1
      decision: challenge
expiring_decision_ttl_seconds: 10
"""


def geom_lines(t, seed, n=3000):
    """Lines of every length class against the scan geometry (4 KB wave
    tiles + 512 B halo, <= 128 lines decided per tile): runs of tiny lines,
    halo-edge lengths, multi-tile lines, literals at random offsets (so they
    straddle tile and halo edges), long headers."""
    import random
    rnd = random.Random(seed)
    toks = [b"needle", b"haystack123x", b"haystack12", b"FooBar", b"fOOBAR", b"sitelit", b"123z", b"alphagammadelta",
            b"omegaa", b"needle7", b"GET /a"]
    out = []
    i = 0
    while i < n:
        kind = rnd.random()
        if kind < 0.05:  # a run of tiny lines (> 128 per tile)
            for _ in range(rnd.randint(150, 400)):
                out.append(b"%d 9.9.9.%d G h G /a" % (t, rnd.randint(0, 9)))
            i += 1
            continue
        if kind < 0.5:
            size = rnd.randint(40, 300)
        elif kind < 0.75:
            size = rnd.randint(300, 800)
        elif kind < 0.95:
            size = rnd.randint(800, 9000)
        else:
            size = rnd.randint(4000, 12000)
        host = rnd.choice([b"h.com", b"x.org", b"h.com", b"y" * rnd.randint(1, 700)])
        m = rnd.choice([b"GET", b"POST"])
        head = b"%d 10.0.%d.%d %s %s %s /a" % (t, rnd.randint(0, 3), rnd.randint(0, 50), m, host, m)
        body = bytearray(rnd.choice(b"abcdefghij klmnop0123456789/") for _ in range(max(0, size - len(head))))
        for _ in range(rnd.randint(0, 4)):
            tok = rnd.choice(toks)
            p = rnd.randint(0, max(0, len(body) - len(tok)))
            body[p:p + len(tok)] = tok
        out.append(head + bytes(body))
        i += 1
    return b"\n".join(out) + b"\n"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tile_geometry(engine, seed):
    t = 1700000000
    pair = Pair(GEOM_CFG, engine)
    data = geom_lines(t, seed)
    pair.feed(data, t * S)
    # same bytes shifted by a few bytes: every literal lands on other tile offsets
    pair.feed(b"\n" * (seed * 7) + data, t * S)
    pair.compare_state(["10.0.0.1", "10.0.1.2", "9.9.9.1"])


def overflow_past_line_cap_lines(t, shift):
    """A 4 KB scan tile whose last line starts after more than kLineCap (128)
    other lines and overflows its hit slots: its IP field holds an
    equivalent rule's literal ("needle", not in rest), and its rest -- in the
    halo, so the scan pass verifies those hits first -- holds five hits of
    another literal.  The IP-field hit then lands past the slots, where the
    scan pass's "far from the line start" test must not read the line-start
    array past its kLineCap entries (round-3 advisor finding)."""
    tiny = b"x\n" * 140
    target = b"%d needle GET h.com GET /a FooBar FooBar FooBar FooBar FooBar fOOBAR\n" % t
    start = 4096 - 25 + shift  # the IP field ends just before the tile edge
    filler_len = start - len(tiny) - 1
    head = b"%d 10.0.0.1 GET h.com GET /a " % t
    filler = head + b"a" * (filler_len - len(head)) + b"\n"
    data = tiny + filler + target
    assert data.index(target) == start
    tail = b"%d 10.0.0.2 GET x.org GET /needle%d HTTP/1.1 ua\n" % (t, shift)
    return data + tail * 3


@pytest.mark.parametrize("shift", [0, 3, 9, 17])
def test_overflow_hits_past_line_cap(engine, shift):
    t = 1700000000
    pair = Pair(GEOM_CFG, engine)
    pair.feed(overflow_past_line_cap_lines(t, shift), t * S)
    pair.compare_state(["needle", "10.0.0.1", "10.0.0.2"])


@pytest.mark.parametrize("mask", [0xFF, 0xFFF])
def test_ip_hash_collisions(engine, mask):
    """Distinct IPs forced onto a few 64-bit hash values (test hook): the IP
    table's exact byte compares and the serial collision resolver
    (k_ip_collide) must keep every IP's state separate, across batches."""
    w = W.scaled(W.CFG5, 30_000, n_ips=6_000)
    engine.debug_set_ip_hash_mask(mask)
    try:
        pair = Pair(w.rules_yaml, engine)
        ips = set()
        for b in range(3):
            data = w.host_lines(b * 10_000, 10_000)
            for ln in data.split(b"\n")[:300]:
                parts = ln.split(b" ")
                if len(parts) > 2:
                    ips.add(parts[1].decode())
            pair.feed(data, w.now_ns(b * 10_000, 10_000))
        pair.compare_state(sorted(ips)[:60])
    finally:
        engine.debug_set_ip_hash_mask(0)


@pytest.mark.parametrize("wl,world,copy", [(("cfg5", 3000), 2, True), (("cfg3", 2000), 3, True), (("cfg3", 2000), 3, False),
                                           (("cfg5", 3000), 2, False)])
def test_sharded_engines_match_single_process(wl, world, copy):
    """The multi-GPU path on one GPU: `world` engines as threads (ThreadMesh),
    each matching its chunk, rate limits sharded by IP hash with the real
    bjx_events_pack / bjx_apply_events / bjx_finish_batch (copy=False: the
    trips-only return, bjx_apply_events_trips / bjx_finish_batch_trips).
    Bit-exact against one oracle over the stream, and each IP's state lives on
    exactly one engine."""
    import threading

    import torch

    from banjax_amd import Ruleset
    from types import SimpleNamespace

    from banjax_amd.distributed import ThreadMesh, merge_rank_bans, sharded_batch
    from banjax_amd.regex_rate_limiter import DynamicDecisionLists
    n_chunks, per = 2 * world, 8000
    w = W.scaled(W.ALL[wl[0]], per * n_chunks, n_ips=wl[1])
    cfg = Config.from_yaml(w.rules_yaml)
    chunks = [w.host_lines(k * per, per) for k in range(n_chunks)]
    dev = torch.device("cuda", 0)
    engines = [Engine(0) for _ in range(world)]
    mesh = ThreadMesh(world)
    got, errs, bans = {}, [], {}

    def run(r):
        try:
            rs = Ruleset(cfg)
            engines[r].set_decision_lists(cfg.decision_entries)
            engines[r].set_ban_options(cfg.expiring_decision_ttl_seconds)
            ex = mesh.rank(r, dev)
            for step in range(n_chunks // world):
                k = step * world + r
                t = torch.frombuffer(bytearray(chunks[k]), dtype=torch.uint8).to(dev)
                out = sharded_batch(engines[r], rs, w.now_ns(0, per), t.data_ptr(), len(chunks[k]), ex,
                                    copy_results=copy, emit_bans=True)
                trips = [SimpleNamespace(line_offset=x.line_offset, line_len=x.line_len, ip_off=x.ip_off,
                                         ip_len=x.ip_len, host_off=x.host_off, host_len=x.host_len) for x in out.trips]
                bans[k] = (engines[r].bans(), trips, chunks[k])
                got[k] = ([[x.line_idx, x.rule_idx, x.rule_pos, x.skip_host, x.seen_ip, x.match_type, x.exceeded]
                           for x in out.results] if copy else None, [(x.line_idx, x.rule_idx) for x in out.trips],
                          bytes(out.line_flags) if copy else None)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            mesh.barrier.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    oc = oracle_config(cfg)
    st = O.State()
    n_trips = 0
    for k, data in enumerate(chunks):
        oflags, ores, _ = st.consume(oc, data, w.now_ns(0, per), cap=(data.count(b"\n") + 1) * (len(cfg.all_rules()) + 1))
        exp = [[r.line_idx, r.rule_id, r.rule_pos, r.skip_host, r.seen_ip, r.match_type, r.exceeded] for r in ores]
        results, trips, flags = got[k]
        if copy:
            assert list(flags) == oflags
            assert results == exp, "chunk %d" % k
        assert trips == [(r[0], r[1]) for r in exp if r[6]], "chunk %d" % k
        n_trips += len(trips)
    assert n_trips > 0
    # device decision emission, merged over the ranks of each step
    dl, blog = DynamicDecisionLists(), []
    for step in range(n_chunks // world):
        recs, log = merge_rank_bans([bans[step * world + r] for r in range(world)])
        for ip, host, d, exp_ns, _, _ in recs:
            dl.update(ip.decode(), exp_ns, d, False, host.decode())
        blog += ["%d %s" % (kind - 1, line.decode()) for kind, line in log]
    assert len(dl.expiring) == st.decisions_len()
    for ip, d in dl.expiring.items():
        assert tuple(st.decision(ip)[:3]) == (d.decision, d.expires_ns, d.domain), ip
    assert blog == [ln for ln in st.ban_log().split("\n") if ln]
    assert sum(e.state_len() for e in engines) == len(st)
    names = sorted(set(r.rule for r in cfg.all_rules()))
    for ln in chunks[0].split(b"\n")[:40]:
        ip = ln.split(b" ")[1]
        for nm in names:
            have = [e.state_get(ip, nm) for e in engines]
            exp = st.get(ip, nm)
            assert [h for h in have if h is not None] == ([exp] if exp is not None else [])
    for e in engines:
        e.close()


@pytest.mark.parametrize("n_parts,trips_only", [(256, False), (7, True), (1, False)])
def test_partition_many_owners_one_engine(n_parts, trips_only):
    """bjx_events_partition / bjx_events_pack with up to 256 owners (many
    distinct owners in every wave of k_pack), the packed records fed straight
    back into the same engine as n_parts "sources": every IP lives in exactly
    one owner segment, in line order, so Apply over the segments in owner
    order gives the reference's outcomes.  Bit-exact against the oracle, over
    the outcome-byte and the trip-list returns."""
    import torch

    w = W.scaled(W.CFG3, 6000, n_ips=3000)
    cfg = Config.from_yaml(w.rules_yaml)
    rs = Ruleset(cfg)
    eng = Engine(0)
    eng.set_decision_lists(cfg.decision_entries)
    oc = oracle_config(cfg)
    st = O.State()
    dev = torch.device("cuda", 0)
    for b in range(2):
        data = w.host_lines(b * 3000, 3000)
        now = w.now_ns(b * 3000, 3000)
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        eng.match(rs, now, t.data_ptr(), len(data), copy_results=not trips_only)
        send = eng.events_partition(n_parts)
        assert sum(c[0] > 0 for c in send) > min(n_parts, 100) // 2
        tl, te, tb = (sum(c[i] for c in send) for i in range(3))
        lines = torch.empty(max(1, tl * 16), dtype=torch.uint8, device=dev)
        events = torch.empty(max(1, te * 4), dtype=torch.uint8, device=dev)
        ipb = torch.empty(max(1, tb), dtype=torch.uint8, device=dev)
        eng.events_pack(lines.data_ptr(), events.data_ptr(), ipb.data_ptr())
        if trips_only:
            base, acc = [], 0
            for c in send:
                base.append(acc)
                acc += c[1]
            tr = torch.empty(max(1, te) * 4, dtype=torch.uint8, device=dev)
            cnt = eng.apply_events_trips(rs, lines.data_ptr(), events.data_ptr(), ipb.data_ptr(), send, base, tr.data_ptr())
            nt = sum(cnt)
            if nt:
                # a list naming one event twice is refused (it would duplicate a trip)
                dup = torch.cat([tr[:nt * 4], tr[:4]])
                with pytest.raises(RuntimeError, match="more than once"):
                    eng.finish_trips(dup.data_ptr(), nt + 1)
            out = eng.finish_trips(tr.data_ptr(), nt)
        else:
            o = torch.empty(max(1, te), dtype=torch.uint8, device=dev)
            eng.apply_events(rs, lines.data_ptr(), events.data_ptr(), ipb.data_ptr(), send, o.data_ptr())
            out = eng.finish(o.data_ptr(), copy_results=True)
        _, ores, _ = st.consume(oc, data, now, cap=(data.count(b"\n") + 1) * (len(cfg.all_rules()) + 1))
        exp = [[r.line_idx, r.rule_id, r.rule_pos, r.skip_host, r.seen_ip, r.match_type, r.exceeded] for r in ores]
        if not trips_only:
            assert [[x.line_idx, x.rule_idx, x.rule_pos, x.skip_host, x.seen_ip, x.match_type, x.exceeded]
                    for x in out.results] == exp
        assert [(x.line_idx, x.rule_idx) for x in out.trips] == [(r[0], r[1]) for r in exp if r[6]]
    assert sum(r[6] for r in exp) > 0
    assert eng.state_len() == len(st)
    eng.close()


@pytest.mark.parametrize("budget,slot_cache", [(1, 1), (97, 1), (5000, 1), (1, 0), (97, 0)])
def test_table_overflow_rollback(engine, budget, slot_cache):
    """The IP and state tables claim at most `budget` new entries in a batch's
    first claim launch (test hook): every batch overflows, rolls its claims
    back and claims again - results stay bit-exact across batches, with the
    state-slot cache on and off."""
    w = W.scaled(W.CFG5, 24_000, n_ips=8_000)
    engine.debug_set_claim_budget(budget)
    engine.debug_set_slot_cache(slot_cache)
    try:
        pair = Pair(w.rules_yaml, engine)
        ips = set()
        for b in range(3):
            data = w.host_lines(b * 8_000, 8_000)
            for ln in data.split(b"\n")[:200]:
                parts = ln.split(b" ")
                if len(parts) > 2:
                    ips.add(parts[1].decode())
            pair.feed(data, w.now_ns(b * 8_000, 8_000))
        pair.compare_state(sorted(ips)[:60])
    finally:
        engine.debug_set_claim_budget(0)
        engine.debug_set_slot_cache(-1)


def test_shared_patterns_across_rules(engine):
    """Rules that repeat one pattern (on several hosts, and as a global) under
    different names, limits, decisions and hosts_to_skip: the device runs one
    automaton per pattern (engine.hip `canon`), while results, state keys and
    trips stay per rule (regex_rate_limiter.go:175-211, rate_limit.go:37-78)."""
    pats = [r"(GET|POST) \S+ (GET|POST) \/admin\/", r"(?i)union.+select", r"^GET \S+ GET \/api\/[0-9]+ ",
            r"\/static\/(js|css)\/", r".*blockme.*"]
    hosts = ["h%d.example.com" % i for i in range(6)]
    decs = ["challenge", "nginx_block", "iptables_block"]
    rnd = random.Random(21)
    out = ["regexes_with_rates:"]
    for k, p in enumerate(pats[:3]):
        out.append("  - rule: 'g%d'\n    regex: '%s'\n    interval: 2\n    hits_per_interval: %d\n    decision: %s\n"
                   "    hosts_to_skip:\n      h1.example.com: true" % (k, p.replace("'", "''"), k, decs[k % 3]))
    out.append("per_site_regexes_with_rates:")
    for hi, h in enumerate(hosts[:5]):
        out.append("  %s:" % h)
        for k, p in enumerate(pats):
            if (hi + k) % 4 == 3:
                continue
            out.append("    - rule: '%s'\n      regex: '%s'\n      interval: %d\n      hits_per_interval: %d\n"
                       "      decision: %s" % ("s%d" % k if hi % 2 else "%s r%d" % (h, k), p.replace("'", "''"),
                                              1 + hi, (hi * k) % 3, decs[(hi + k) % 3]))
    pair = Pair("\n".join(out) + "\n", engine)
    uris = ["/admin/x", "/api/12 ", "/static/js/a.js", "/q?UNION%20x%20select", "/blockme", "/admin", "/api/x", "/"]
    base = 1700000000
    for b in range(2):
        lines = []
        for j in range(6000):
            m = rnd.choice(["GET", "POST"])
            lines.append("%.3f 10.0.%d.%d %s %s %s %s HTTP/1.1 UA-%d\n" % (
                base + b * 3 + j * 0.0004, rnd.randrange(4), rnd.randrange(8), m, rnd.choice(hosts), m,
                rnd.choice(uris) + rnd.choice(["", " ", "x"]), j % 7))
        pair.feed("".join(lines).encode(), (base + b * 3 + 3) * S)
    pair.compare_state(["10.0.%d.%d" % (a, c) for a in range(4) for c in range(8)])


def test_bounded_lead_rules(engine):
    """Rules whose matches begin a bounded distance before their literals
    (tests/test_lead_cpu.py): their DFA jobs start near the first literal hit.
    Lines with 0..12 hits (past 4 the hit slots overflow and the first hit of
    any literal bounds the start), cut runes and non-ASCII bytes before hits."""
    from tests.test_lead_cpu import CASES
    rnd = random.Random(17)
    pats = [p for p, _, _ in CASES]
    yaml_rules = ["regexes_with_rates:"]
    for i, p in enumerate(pats):
        yaml_rules.append("  - rule: 'l%d'\n    regex: '%s'\n    interval: 1\n    hits_per_interval: 1000000\n"
                          "    decision: challenge" % (i, p.replace("'", "''")))
    pair = Pair("\n".join(yaml_rules) + "\n", engine)
    frags = [b"a", b"b", b"x", b"12", b" ", b"=", b"\xc3\xa9", b"\xc5\xbf", b"\xe2\x84\xaa", b"\xff", b"S", b"s",
             b"crapy", b"CRAPY", b"mechanize", b"abcd", b"=token", b"wxyz", b"abwxyz1", b"Macintosh", b"Firefox/9",
             b"Firefox/", b"qqqqqqqqqqqqqqqqqqqqqqqqqqqqqq"]
    lines = []
    for j in range(4000):
        body = b"".join(rnd.choice(frags) for _ in range(rnd.randrange(0, 40)))
        lines.append(b"1700000000 9.9.9.%d GET h%d.com " % (j % 250, j % 7) + body)
    pair.feed(b"\n".join(lines) + b"\n", 1700000000 * S)


def test_dfa_self_loop_acceleration(engine):
    """States left by at most 3 ASCII bytes (a `.*` waiting for a literal) are
    skipped 16 B at a time (engine.hip dfa_text / Bind::accel): long texts with
    sparse escape bytes at every offset of a 16 B chunk, non-ASCII bytes, cut
    runes and matches ending at the last byte."""
    rnd = random.Random(23)
    pats = [r"Macintosh.*Firefox/\d+", r"ab.*cde.*f", r"[^z]*z.{3}", r"q.*[xy]\d", r"(?i)start.*stop$", r"wq.*é",
            r"k.*\bend\b", r"zz[^\n]*zz"]
    yaml_rules = ["regexes_with_rates:"]
    for i, p in enumerate(pats):
        yaml_rules.append("  - rule: 'a%d'\n    regex: '%s'\n    interval: 1\n    hits_per_interval: 1000000\n"
                          "    decision: challenge" % (i, p.replace("'", "''")))
    pair = Pair("\n".join(yaml_rules) + "\n", engine)
    fill = [b"m", b"n", b"o", b"p", b" ", b"-", b"/", b"1"]
    rare = [b"Macintosh", b"Firefox/7", b"Firefox/", b"ab", b"cde", b"f", b"z", b"zz", b"q", b"x", b"y9", b"START",
            b"stop", b"wq", b"\xc3\xa9", b"\xc3", b"\xff", b"k", b"end", b" end "]
    lines = []
    for j in range(3000):
        parts = []
        for _ in range(rnd.randrange(0, 12)):
            parts.append(b"".join(rnd.choice(fill) for _ in range(rnd.randrange(0, 300))))
            parts.append(rnd.choice(rare))
        lines.append(b"1700000000 9.9.9.%d GET h%d.com " % (j % 250, j % 7) + b"".join(parts))
    pair.feed(b"\n".join(lines) + b"\n", 1700000000 * S)


@pytest.mark.parametrize("name,n_lines,batches", [("cfg3", 60_000, 2), ("cfg5", 40_000, 2), ("cfg1", 100_000, 2),
                                                  ("cfg5h", 60_000, 2)])
def test_workload_trips_only(engine, name, n_lines, batches):
    """The bench's path: no RuleResult copies (the events alone feed the
    claims and the trips).  States, decisions and the ban log (every trip, in
    order) against the oracle."""
    w = W.scaled(W.ALL[name], n_lines, n_ips=min(W.ALL[name].n_ips, n_lines // 3 + 1))
    pair = Pair(w.rules_yaml, engine)
    per = (n_lines + batches - 1) // batches
    ips = set()
    for b in range(batches):
        first, cnt = b * per, min(per, n_lines - b * per)
        data = w.host_lines(first, cnt)
        for ln in data.split(b"\n")[:200]:
            parts = ln.split(b" ")
            if len(parts) > 2:
                ips.add(parts[1].decode())
        pair.feed(data, w.now_ns(first, cnt), want_results=False)
    pair.compare_state(sorted(ips)[:100])


@pytest.mark.parametrize("budget", [1, 97])
def test_trips_only_claim_rollback(engine, budget):
    """The claims' rollback paths (both tables) under the claim-budget hook,
    on the trip-only path."""
    w = W.scaled(W.CFG5, 24_000, n_ips=8_000)
    engine.debug_set_claim_budget(budget)
    try:
        pair = Pair(w.rules_yaml, engine)
        for b in range(3):
            pair.feed(w.host_lines(b * 8_000, 8_000), w.now_ns(b * 8_000, 8_000), want_results=False)
        pair.compare_state()
    finally:
        engine.debug_set_claim_budget(0)


def short_lines(t, n, k):
    """n lines of ~40 bytes: far more lines per byte (and per scan tile) than
    the batches before them."""
    return b"".join(b"%d 10.%d.0.%d GET s.com GET /%d h\n" % (t, k % 7, i % 50, i % 13) for i in range(n))


def test_short_line_batches(engine):
    """Batches of ordinary lines, then a batch of short lines (over 100 lines
    per 4 KB scan tile), then ordinary lines again: every batch matches the
    oracle and the per-line arrays follow the line counts."""
    w = W.scaled(W.CFG3, 60_000, n_ips=3_000)
    t = w.now_ns(0, 1) // S
    pair = Pair(w.rules_yaml, engine)
    for b in range(2):
        pair.feed(w.host_lines(b * 20_000, 20_000), w.now_ns(b * 20_000, 20_000))
    pair.feed(short_lines(t, 30_000, 1), t * S)
    pair.feed(w.host_lines(40_000, 20_000), w.now_ns(40_000, 20_000))
    pair.compare_state(["10.1.0.1", "10.1.0.2"])


def test_compact_trips_match_full(engine):
    """BJX_TRIPS_COMPACT words carry each trip's line offset and rule index,
    in reference order, equal to the full bjx_trip records of the same batch
    on the same state."""
    w = W.scaled(W.CFG5, 40_000, n_ips=4_000)
    rs = Ruleset(Config.from_yaml(w.rules_yaml))
    data = w.host_lines(0, 40_000)
    now = w.now_ns(0, 40_000)
    engine.state_clear()
    full = engine.process(rs, data, now)
    want = [(t.line_offset, t.rule_idx) for t in full.trips]
    engine.state_clear()
    comp = engine.process(rs, data, now, compact_trips=True)
    words = comp.trips_compact()
    got = [(int(x) >> 24, int(x) & 0xFFFFFF) for x in words]
    engine.state_clear()
    assert comp.n_trips == full.n_trips == len(want) > 100
    assert got == want
    for off, _ in got[:50]:  # the offset starts a line
        assert off == 0 or data[off - 1:off] == b"\n"


@pytest.mark.parametrize("rec16", [0, 1])
def test_event_record_forms(engine, rec16, monkeypatch):
    """The event sort carries 12-B records (engine_types.h EvRec12: timestamps
    within 2^43 ns of the batch's clock); a batch whose events lie 3 h past
    its clock is claimed again and sorted in the 16-B form, and BJX_REC16=1
    forces that form throughout.  Results stay bit-exact against the oracle
    through state carried across the batches."""
    if rec16:
        monkeypatch.setenv("BJX_REC16", "1")
    w = W.scaled(W.CFG3, 40_000, n_ips=2_000)
    pair = Pair(w.rules_yaml, engine)
    pair.feed(w.host_lines(0, 10_000), w.now_ns(0, 10_000))
    pair.feed(w.host_lines(10_000, 10_000), w.now_ns(10_000, 10_000) - 3 * 3600 * S)
    pair.feed(w.host_lines(20_000, 10_000), w.now_ns(20_000, 10_000), want_results=False)
    pair.feed(w.host_lines(30_000, 10_000), w.now_ns(30_000, 10_000) - 3 * 3600 * S, want_results=False)
    pair.compare_state()


def test_lines2_wide_masks(engine):
    """k_lines2 with 2-word position masks and literal ids past 32: a host of
    12 site rules plus 110 global rules (positions up to 121), with ALWAYS,
    anchored, no-literal and hosts_to_skip rules past position 64 and lines
    whose literal hits overflow the scan's 4 slots.  Bit-exact against the
    oracle, and the window kernel is the one that ran."""
    rnd = random.Random(41)
    decs = ["challenge", "nginx_block", "iptables_block"]
    out = ["regexes_with_rates:"]
    for k in range(110):
        if k in (3, 70, 101):
            p = r".*"
        elif k % 17 == 5:
            p = r"^GET \S+ GET \/q%d\/" % k
        elif k % 23 == 7:
            p = r"(GET|POST) \S+ (GET|POST) \/[a-z]%d[0-9]+" % k
        else:
            p = r"\/p%03d\/[a-z]+" % k if k % 2 else r"tok%03dx" % k
        skip = "\n    hosts_to_skip:\n      s.example.com: true" if k in (66, 90, 101) else ""
        out.append("  - rule: 'g%d'\n    regex: '%s'\n    interval: %d\n    hits_per_interval: %d\n    decision: %s%s"
                   % (k, p, 1 + k % 3, k % 4, decs[k % 3], skip))
    out.append("per_site_regexes_with_rates:")
    out.append("  s.example.com:")
    for k in range(12):
        out.append("    - rule: 's%d'\n      regex: '%s'\n      interval: 2\n      hits_per_interval: 1\n      decision: %s"
                   % (k, r"\/site%d\/" % k, decs[k % 3]))
    pair = Pair("\n".join(out) + "\n", engine)
    hosts = ["s.example.com", "o.example.com"]
    frags = ["/p%03d/ab" % k for k in range(1, 110, 2)] + ["tok%03dx" % k for k in range(0, 110, 2)] + \
            ["/q%d/" % k for k in range(5, 110, 17)] + ["/b%d77" % k for k in range(7, 110, 23)] + \
            ["/site%d/" % k for k in range(12)] + ["/none", "zz"]
    base = 1700000000
    for b in range(2):
        lines = []
        for j in range(5000):
            n_frag = rnd.choice([0, 1, 1, 2, 3, 6, 9])
            uri = "".join(rnd.choice(frags) for _ in range(n_frag)) or "/"
            lines.append("%.3f 10.1.%d.%d GET %s GET %s HTTP/1.1 UA\n" % (
                base + b * 2 + j * 0.0003, rnd.randrange(4), rnd.randrange(16), rnd.choice(hosts), uri))
        pair.feed("".join(lines).encode(), (base + b * 2 + 2) * S)
        assert pair.engine.line_kernel()[0] == "k_lines2"
    pair.compare_state(["10.1.%d.%d" % (a, c) for a in range(4) for c in range(16)])


@pytest.mark.parametrize("switch,name", [("BJX_NO_LINES2", "cfg3"), ("BJX_NO_PLAN_LDS", "cfg3"), ("BJX_NO_HOST_LDS", "cfg3"),
                                         ("BJX_NO_PLAN", "cfg2"), ("BJX_NO_DFA_SKIP", "cfg5")])
def test_fallback_paths(switch, name, monkeypatch):
    """The bind-time switches that force a fallback path (the per-line
    kernel k_lines, plan tables in HBM, the host dictionary in HBM, the rule
    walk without plans, DFA jobs from rest[0]): the paths a ruleset too large
    for the fast tables takes, bit-exact against the oracle."""
    monkeypatch.setenv(switch, "1")
    eng = Engine(0)
    w = W.scaled(W.ALL[name], 20_000, n_ips=4_000)
    pair = Pair(w.rules_yaml, eng)
    for b in range(2):
        pair.feed(w.host_lines(b * 10_000, 10_000), w.now_ns(b * 10_000, 10_000))
    if switch == "BJX_NO_LINES2":
        assert eng.line_kernel()[0] == "k_lines"
    pair.compare_state([ln.split(b" ")[1].decode() for ln in w.host_lines(0, 50).split(b"\n")[:50] if ln])
    eng.close()


@pytest.mark.parametrize("name,rec16,check", [("cfg3", 0, 0), ("cfg5", 0, 0), ("cfg1", 0, 0), ("cfg3", 1, 0), ("cfg1", 0, 1)])
def test_two_level_grouping(engine, name, rec16, check, monkeypatch):
    """The rate-limit stage's two-level grouping (engine.hip k_bucket_apply:
    the event sort on the state slot's high 16 bits, then each bucket ranked by
    its low bits in LDS) forced on test-sized batches with BJX_SORT2=2, for both
    record forms; cfg1's Zipf IPs overflow buckets, whose events take the full
    sort on their own.  Bit-exact against the oracle's sequential Apply
    (rate_limit.go:37-78) through state carried across the batches.  With
    BJX_CHECK=1 the engine also verifies, per batch, that every bucket-sorted
    outcome is written exactly once (k_bucket_apply, and k_apply + k_big_outs
    for the overflowing buckets) and that the sorted records are a permutation."""
    monkeypatch.setenv("BJX_SORT2", "2")
    if check:
        monkeypatch.setenv("BJX_CHECK", "1")
    if rec16:
        monkeypatch.setenv("BJX_REC16", "1")
    engine.state_clear()
    w = W.scaled(W.ALL[name], 60_000, n_ips=3_000)
    pair = Pair(w.rules_yaml, engine)
    for b in range(3):
        pair.feed(w.host_lines(b * 20_000, 20_000), w.now_ns(b * 20_000, 20_000))
        assert engine.scan_stats()["grouping"] >= 1
    pair.compare_state([ln.split(b" ")[1].decode() for ln in w.host_lines(0, 50).split(b"\n")[:50] if ln])
