"""Pin the oracle (oracle/bjx_oracle.c) against the reference's own tests.

Each test restates a reference Go test at the consumeLine boundary with the
injected clock now_ns (the Go tests use time.Now(); every line they feed is
<= 10 s old or in the future, so OldLine never fires there either).
"""
import random

import pytest

from oracle import oracle as O

S = 1_000_000_000


def line(ts, rest):
    return ("%f %s\n" % (ts, rest)).encode()


def test_consume_line_sequence():
    """regex_rate_limiter_test.go:77-260 TestConsumeLine."""
    cfg = O.Config()
    cfg.add_rule("rule1", r"GET example\.com GET .*", 5 * S, 2, O.NGINX_BLOCK)
    cfg.add_rule("rule2", r"POST .*", 5 * S, 1, O.CHALLENGE)
    cfg.add_rule("instant block", r".*blockme.*", 1 * S, 0, O.NGINX_BLOCK, site="per-site.com")
    st = O.State()
    t0 = 1700000000.123456
    now = int(t0 * 1e9)
    ua = "AppleWebKit/537.36 (KHTML, like Gecko) Chrome/51.0.2704.103 Safari/537.36 -"
    get = "1.2.3.4 GET example.com GET /whatever HTTP/1.1 " + ua
    post = "1.2.3.4 POST example.com POST /whatever HTTP/1.1 " + ua

    st.consume(cfg, line(t0, get), now)
    assert st.get("1.2.3.4", "rule1")[0] == 1
    assert st.banned_ip() == ""
    st.consume(cfg, line(t0 + 4, get), now)
    assert st.get("1.2.3.4", "rule1")[0] == 2
    assert st.banned_ip() == ""
    st.consume(cfg, line(t0 + 5.5, get), now)
    assert st.get("1.2.3.4", "rule1")[0] == 1
    assert st.banned_ip() == ""
    st.consume(cfg, line(t0 + 6.5, post), now)
    assert st.get("1.2.3.4", "rule1")[0] == 1
    assert st.get("1.2.3.4", "rule2")[0] == 1
    assert st.banned_ip() == ""
    st.consume(cfg, line(t0 + 7.0, post), now)
    assert st.get("1.2.3.4", "rule1")[0] == 1
    assert st.get("1.2.3.4", "rule2")[0] == 0
    assert st.banned_ip() == "1.2.3.4"
    st.consume(cfg, line(t0 + 20, "1.6.6.6 GET per-site.com GET /blockme/?a HTTP/1.1 " + ua), now)
    assert st.get("1.6.6.6", "instant block") is not None
    st.consume(cfg, line(t0 + 22, "1.6.6.7 GET no-per-site.com GET /blockme/?a HTTP/1.1 " + ua), now)
    assert st.get("1.6.6.7", "instant block") is None and len(st) == 2


def test_consume_line_hosts_to_skip():
    """regex_rate_limiter_test.go:262-297 TestConsumeLineHostsToSkip."""
    cfg = O.Config()
    cfg.add_rule("rule1", r"^GET https?:\/\/\.*", 5 * S, 2, O.NGINX_BLOCK, hosts_to_skip=["skiphost.com"])
    st = O.State()
    t0 = 1700000000.5
    flags, res, _ = st.consume(cfg, line(t0, "1.2.3.4 GET skiphost.com GET /whatever HTTP/1.1 x"), int(t0 * 1e9))
    assert len(st) == 0
    # rest is "GET skiphost.com GET ..." -> "^GET https?://" does not match: no RuleResult at all
    assert res == []
    # beyond the reference test: "GET skiphost.com GET http://x" still fails
    # the anchored "^GET https?://" (rest starts at the first method), so no
    # RuleResult and no state either
    flags, res, _ = st.consume(cfg, line(t0, "1.2.3.4 GET skiphost.com GET http://x HTTP/1.1 x"), int(t0 * 1e9))
    assert res == [] and flags == [0] and len(st) == 0
    flags, res, _ = st.consume(cfg, line(t0, "1.2.3.4 GET https://a.b GET /x HTTP/1.1 x"), int(t0 * 1e9))
    assert len(res) == 1 and res[0].skip_host == 0 and len(st) == 1


def test_per_site_regex_stress_structure():
    """regex_rate_limiter_test.go:299-365 TestPerSiteRegexStress (structural;
    the reference draws unseeded gofakeit data, here a seeded equivalent)."""
    rnd = random.Random(7)
    n = 1500
    cfg = O.Config()
    domains, paths = [], []
    for i in range(n):
        d = "%s%d.%s" % (rnd.choice(["acme", "shop", "news", "blog"]), i, rnd.choice(["com", "org", "net"]))
        p = "/%s/%d" % (rnd.choice(["a", "img", "api"]), rnd.randrange(10 ** 6))
        cfg.add_rule("rule%d" % i, r"GET %s GET \%s HTTP\/[0-2.]+ .*" % (d.replace(".", r"\."), p),
                     1 * S, 0, O.NGINX_BLOCK)
        domains.append(d)
        paths.append(p)
    st = O.State()
    base = 1700000000
    for j in range(n):
        ip = "%d.%d.%d.%d" % (rnd.randrange(1, 255), rnd.randrange(256), rnd.randrange(256), rnd.randrange(256))
        ln = "%f %s GET %s GET %s HTTP/2.0 Mozilla/5.0 (X11)\n" % (float(base + j), ip, domains[j], paths[j])
        st.consume(cfg, ln.encode(), (base + j) * S)
        got = st.get(ip, "rule%d" % j)
        assert got is not None and got[0] == 0
        assert st.banned_ip() == ip


@pytest.mark.parametrize("pat,text,exp", [
    (r"Macintosh.*Firefox/\d+", "Mozilla/5.0 (Macintosh; Intel Mac OS X 10.15; rv:149.0) Gecko/20100101 Firefox/149.0", True),
    (r"Macintosh.*Firefox/\d+", "Mozilla/5.0 (Windows NT 10.0; Win64; x64; rv:149.0) Gecko/20100101 Firefox/149.0", False),
    (r"(?i)scrapy|mechanize", "Scrapy/2.11.2 (+https://scrapy.org)", True),
    (r"(?i)scrapy|mechanize", "Python-Mechanize/0.4.9", True),
    (r"(?i)scrapy|mechanize", "Mozilla/5.0 (compatible; Googlebot/2.1)", False),
])
def test_user_agent_regex_known_answers(pat, text, exp):
    """user_agent_decision_test.go:28-45 (Go regexp known answers)."""
    assert O.Regex(pat).match(text) is exp


def test_invalid_regex_is_a_compile_error():
    """user_agent_decision_test.go:47-50 and config.go:110-113."""
    assert O.compile_error("(?invalid") == "error parsing regexp: invalid or unsupported Perl syntax: `(?in`"
    cfg = O.Config()
    with pytest.raises(ValueError):
        cfg.add_rule("bad", "(?invalid", S, 0, O.ALLOW)


def test_allow_lists_exempt():
    """banjax_integration_test.go:387-407 TestRegexesWithRatesAllowList with the
    fixtures/banjax-config-test.yaml decision lists."""
    cfg = O.Config()
    cfg.add_rule("instant block_local", ".*block_local", S, 0, O.NGINX_BLOCK, site="localhost:8081")
    cfg.add_rule("instant block", ".*blockme.*", S, 0, O.NGINX_BLOCK)
    cfg.add_decision_ip(O.ALLOW, "20.20.20.20")
    for ip in ("8.8.8.8", "60.60.60.60", "192.168.1.0/24"):
        cfg.add_decision_ip(O.CHALLENGE, ip)
    cfg.add_decision_ip(O.ALLOW, "90.90.90.90", site="localhost:8081")
    cfg.add_decision_ip(O.ALLOW, "171.171.171.0/24", site="localhost:8081")
    st = O.State()
    t = 1700000000.0
    buf = b"".join([
        line(t, "171.171.171.171 GET localhost:8081 GET /block_local HTTP/1.1 Go"),
        line(t, "20.20.20.20 GET localhost:8081 GET /blockme/ HTTP/1.1 Go"),
        line(t, "171.171.172.1 GET localhost:8081 GET /block_local HTTP/1.1 Go"),
        line(t, "171.171.171.9 GET other.com GET /blockme/ HTTP/1.1 Go"),
    ])
    flags, res, _ = st.consume(cfg, buf, int(t * 1e9))
    assert flags == [O.LINE_EXEMPTED, O.LINE_EXEMPTED, 0, 0]
    assert [r.exceeded for r in res] == [1, 1]


def test_line_errors_and_old_lines():
    cfg = O.Config()
    cfg.add_rule("all", ".*", S, 100, O.CHALLENGE)
    st = O.State()
    t = 1700000000.0
    now = int(t * 1e9)
    buf = b"\n" + b"x\n" + b"1.5 1.2.3.4\n" + b"abc 1.2.3.4 GET h GET / x\n" + b"1700000000 1.2.3.4 GET\n" \
        + line(t - 11, "1.2.3.4 GET h GET / x") + line(t - 9, "1.2.3.4 GET h GET / x") + b"1e400 1.2.3.4 GET h x\n"
    flags, res, _ = st.consume(cfg, buf, now)
    assert flags == [1, 1, 1, 1, 1, 2, 0, 1]


# ---- banjax_integration_test.go:293-385: the reference's end-to-end rate-limit
# cases, restated at the consumeLine boundary.  In -standalone-testing mode the
# HTTP server writes one log line per request (internal/http_server.go:150-167,
# workloads.standalone_line) and the tailer consumes it; the HTTP status the
# test asserts comes from the dynamic decision list the trips leave behind
# (Challenge -> 429, NginxBlock -> 403, none -> 200).

def _kat_state(yaml_text):
    from banjax_amd import Config
    from tests.parity import oracle_config
    cfg = Config.from_yaml(yaml_text)
    return oracle_config(cfg), [r.rule for r in cfg.all_rules()]


def _summary(res, names):
    return [(r.line_idx, names[r.rule_id], r.skip_host, r.seen_ip, r.match_type, r.exceeded) for r in res]


FT, OI, II = 0, 1, 2  # RateLimitMatchType: FirstTime, OutsideInterval, InsideInterval


def test_regexes_with_rates_challengeme_and_reload():
    """TestRegexesWithRatesChallengeme (:293-325) with
    fixtures/banjax-config-test.yaml, then the SIGHUP reload to
    fixtures/banjax-config-test-reload.yaml (banjax.go:101-115), which removes
    the rule and clears the dynamic decision lists."""
    import workloads as W
    cfg, names = _kat_state(W.FIXTURE_RULES)
    st = O.State()
    t0 = 1700000000
    # request 1 passes (its own trip lands after the response) ...
    flags, res, _ = st.consume(cfg, W.standalone_line(t0, "9.9.9.9", "/1?challengeme"), t0 * S)
    assert flags == [0]
    assert _summary(res, names) == [(0, "instant challenge", 0, 0, FT, 1)]
    assert st.decision("9.9.9.9") == (O.CHALLENGE, (t0 + 10) * S, "localhost:8081")
    # ... request 2, two seconds later, meets the Challenge: 429
    flags, res, _ = st.consume(cfg, W.standalone_line(t0 + 2, "9.9.9.9", "/2?challengeme"), (t0 + 2) * S)
    assert _summary(res, names) == [(0, "instant challenge", 0, 1, OI, 1)]
    assert st.decision("9.9.9.9")[0] == O.CHALLENGE
    # SIGHUP: the rule is gone and the dynamic lists are cleared: 200, 200
    cfg, names = _kat_state(W.RELOAD_RULES)
    st.decisions_clear()
    for k in (3, 4):
        flags, res, _ = st.consume(cfg, W.standalone_line(t0 + 3, "9.9.9.9", "/%d?challengeme" % k), (t0 + 3) * S)
        assert flags == [0] and res == []
    assert st.decision("9.9.9.9") is None and st.decisions_len() == 0
    # RegexRateLimitStates survives the reload (banjax.go:113-115 keeps regexStates)
    assert st.get("9.9.9.9", "instant challenge") == (0, (t0 + 2) * S)


def test_regexes_with_rates_skip_limit_and_allow_list():
    """TestRegexesWithRates (:327-385) with
    fixtures/banjax-config-test-regex-banner.yaml:63-92."""
    import workloads as W
    cfg, names = _kat_state(W.REGEX_BANNER_RULES)
    st = O.State()
    t0 = 1700000000
    every, get45 = "Challenge all but skip localhost:8081", "All sites/GET: 45 req/60 sec"
    # target 1: `.*` challenges every host but localhost:8081 -> SkipHost, no Apply: 200, 200
    flags, res, _ = st.consume(cfg, W.standalone_line(t0, "10.10.10.10", "/1"), t0 * S)
    assert _summary(res, names) == [(0, every, 1, 0, FT, 0), (0, get45, 0, 0, FT, 0)]
    flags, res, _ = st.consume(cfg, W.standalone_line(t0 + 2, "10.10.10.10", "/2"), (t0 + 2) * S)
    assert _summary(res, names) == [(0, every, 1, 0, FT, 0), (0, get45, 0, 1, II, 0)]
    assert st.decision("10.10.10.10") is None and st.get("10.10.10.10", every) is None
    # target 2: httpStress sends repeat + 1 = 46 requests; the 46th exceeds 45 in 60 s
    buf = W.standalone_line(t0 + 2, "11.11.11.11", "/45in60") * 46
    flags, res, _ = st.consume(cfg, buf, (t0 + 2) * S)
    g = [x for x in _summary(res, names) if x[1] == get45]
    assert len(g) == 46 and g[0][2:] == (0, 0, FT, 0)
    assert all(x[2:] == (0, 1, II, 0) for x in g[1:45]) and g[45][2:] == (0, 1, II, 1)
    assert st.decision("11.11.11.11") == (O.NGINX_BLOCK, (t0 + 12) * S, "localhost:8081")  # -> 403
    flags, res, _ = st.consume(cfg, W.standalone_line(t0 + 4, "11.11.11.11", "/45in60"), (t0 + 4) * S)
    assert [x for x in _summary(res, names) if x[1] == get45] == [(0, get45, 0, 1, II, 0)]
    assert st.get("11.11.11.11", get45) == (1, (t0 + 2) * S)
    # target 3: the same 46 requests from the global allow list: Exempted, no state, 200
    buf = W.standalone_line(t0 + 4, "12.12.12.12", "/45in60-whitelist") * 46
    flags, res, _ = st.consume(cfg, buf, (t0 + 4) * S)
    assert flags == [O.LINE_EXEMPTED] * 46 and res == []
    assert st.get("12.12.12.12", get45) is None and st.decision("12.12.12.12") is None
