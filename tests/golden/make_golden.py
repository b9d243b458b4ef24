"""Generate the golden consumeLine vectors under tests/golden/ (test data).

Each fixture is an input (a config in the reference's YAML schema, log
batches in nginx banjax_format, an injected clock) plus everything the
reference's consumeLine path produces for it (internal/regex_rate_limiter.go:
113-269, internal/rate_limit.go:37-78): per-line Error/OldLine/Exempted, the
RuleResults in reference order, the trips, the final RegexRateLimitStates of
every (ip, rule name) that saw a result, the DynamicDecisionLists the Banner
replay built, and the LogRegexBan lines.

Expected outputs come from oracle/ (the C restatement), which
tests/test_oracle_reference_kat.py pins against the reference's own Go tests
(TestConsumeLine, TestConsumeLineHostsToSkip, TestPerSiteRegexStress,
TestRegexWithRate, the user-agent regexp known answers).  No Go toolchain
exists in this image, so the reference binary cannot produce them directly
(SURVEY.md §8c).

usage: python tests/golden/make_golden.py [NAME ...]
       (rewrites tests/golden/NAME.json.gz, or every fixture without NAME)
"""
from __future__ import annotations

import base64
import gzip
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import workloads as W  # noqa: E402
from banjax_amd import Config  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.parity import oracle_config  # noqa: E402
from tests.test_gpu_parity import EDGE_CFG, GEOM_CFG, edge_lines, geom_lines  # noqa: E402

S = 1_000_000_000

SEQ_CFG = r"""
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
  "per-site.com":
    - decision: nginx_block
      rule: 'instant block'
      regex: '.*blockme.*'
      interval: 1
      hits_per_interval: 0
expiring_decision_ttl_seconds: 10
"""


def seq_batches():
    """regex_rate_limiter_test.go:77-260 TestConsumeLine, as one batch per line."""
    t0 = 1700000000.123456
    ua = "AppleWebKit/537.36 (KHTML, like Gecko) Chrome/51.0.2704.103 Safari/537.36 -"
    get = "1.2.3.4 GET example.com GET /whatever HTTP/1.1 " + ua
    post = "1.2.3.4 POST example.com POST /whatever HTTP/1.1 " + ua
    seq = [(0, get), (4, get), (5.5, get), (6.5, post), (7.0, post),
           (20, "1.6.6.6 GET per-site.com GET /blockme/?a HTTP/1.1 " + ua),
           (22, "1.6.6.7 GET no-per-site.com GET /blockme/?a HTTP/1.1 " + ua)]
    now = int(t0 * 1e9)
    return [(("%f %s\n" % (t0 + dt, rest)).encode(), now) for dt, rest in seq]


def fixture_lines(t):
    """fixtures/banjax-config-test.yaml rules: triggers, exemptions, per-site rule."""
    L = []
    for ip, host, path in [
            ("1.1.1.1", "example.com", "/?allowme=1"), ("1.1.1.1", "example.com", "/blockme"),
            ("2.2.2.2", "localhost:8081", "/a/block_local"), ("2.2.2.2", "localhost:8081", "/challengeme"),
            ("20.20.20.20", "example.com", "/blockme"),            # global allow: exempt
            ("90.90.90.90", "localhost:8081", "/block_local"),     # per-site allow: exempt
            ("90.90.90.90", "example.com", "/blockme"),            # per-site allow for example.com
            ("171.171.171.9", "localhost:8081", "/blockme"),       # per-site CIDR allow
            ("171.171.171.9", "other.org", "/blockme"),            # CIDR only on localhost:8081
            ("8.8.8.8", "example.com", "/challengeme/and/blockme"),
            ("3.3.3.3", "localhost:8081", "/nothing"),
            ("::1", "localhost:8081", "/block_local?challengeme"),
    ]:
        L.append(b"%d.250 %s GET %s GET %s HTTP/1.1 Mozilla/5.0 (X11; Linux x86_64) | 200"
                 % (t, ip.encode(), host.encode(), path.encode()))
    L.append(b"%d.100 4.4.4.4 GET example.com GET /blockme HTTP/1.1 short" % (t - 11))  # OldLine
    L.append(b"not-a-timestamp 4.4.4.4 GET example.com GET /blockme HTTP/1.1 x")        # Error
    L.append(b"%d 4.4.4.4 GET" % t)                                                     # Error
    return b"\n".join(L) + b"\n"


def workload_batches(name, n_lines, batches, n_ips):
    w = W.scaled(W.ALL[name], n_lines, n_ips=n_ips)
    per = (n_lines + batches - 1) // batches
    out = []
    for b in range(batches):
        first, cnt = b * per, min(per, n_lines - b * per)
        out.append((w.host_lines(first, cnt), w.now_ns(first, cnt)))
    return w.rules_yaml, out


ONLY = set(sys.argv[1:])


def run(name, cfg_yaml, batches, note):
    """batches: (log bytes, now_ns) or (log bytes, now_ns, yaml): the third
    form first runs the reference's SIGHUP handler with that config
    (banjax.go:101-115: ConfigHolder.Reload, DynamicDecisionLists.Clear)."""
    if ONLY and name not in ONLY:
        return
    cfg = Config.from_yaml(cfg_yaml)
    oc = oracle_config(cfg)
    st = O.State()
    n_rules = len(cfg.all_rules())
    rule_names = [r.rule for r in cfg.all_rules()]  # ruleset index order: globals, then sites in YAML order
    recs, keys = [], {}
    for data, now, *reload in batches:
        sighup = None
        if reload:
            sighup = reload[0]
            cfg = Config.from_yaml(sighup)
            oc = oracle_config(cfg)
            n_rules = len(cfg.all_rules())
            rule_names = [r.rule for r in cfg.all_rules()]
            st.decisions_clear()
        flags, res, consumed = st.consume(oc, data, now, cap=(data.count(b"\n") + 1) * (n_rules + 1))
        lines = data[:consumed].split(b"\n")
        results = [[r.line_idx, r.rule_id, r.rule_pos, r.skip_host, r.seen_ip, r.match_type, r.exceeded] for r in res]
        for r in res:
            parts = lines[r.line_idx].split(b" ", 2)
            keys[(parts[1], rule_names[r.rule_id])] = None
        rec = {"log_b64": base64.b64encode(data).decode(), "now_ns": now, "consumed": consumed,
               "flags": flags, "results": results,
               "trips": [[r.line_idx, r.rule_id] for r in res if r.exceeded]}
        if sighup is not None:
            rec["sighup_yaml"] = sighup
        recs.append(rec)
    states = []
    for ip, nm in keys:
        g = st.get(ip, nm)
        states.append([base64.b64encode(ip).decode(), nm, None if g is None else g[0], None if g is None else g[1]])
    decisions = []
    for ip in sorted({k[0] for k in keys}):
        d = st.decision(ip)
        if d is not None:
            decisions.append([base64.b64encode(ip).decode(), d[0], d[1], d[2]])
    fx = {"name": name, "note": note, "config_yaml": cfg_yaml, "batches": recs, "state_len": len(st),
          "states": states, "decisions": decisions, "decisions_len": st.decisions_len(),
          "banned_ip": st.banned_ip(), "ban_log": [l for l in st.ban_log().split("\n") if l]}
    path = os.path.join(HERE, name + ".json.gz")
    with gzip.open(path, "wt", encoding="utf-8") as f:
        json.dump(fx, f, separators=(",", ":"), sort_keys=True)
    print("%-22s %6d B  %d batches, %d results, %d trips" % (
        name, os.path.getsize(path), len(recs), sum(len(r["results"]) for r in recs),
        sum(len(r["trips"]) for r in recs)))


def integration_challengeme(t):
    """banjax_integration_test.go:293-325 TestRegexesWithRatesChallengeme: the
    standalone-testing log lines (internal/http_server.go:150-167) of its
    requests, then the reload that removes the rule."""
    L = W.standalone_line
    return [(L(t, "9.9.9.9", "/1?challengeme"), t * S),
            (L(t + 2, "9.9.9.9", "/2?challengeme"), (t + 2) * S),
            (L(t + 3, "9.9.9.9", "/3?challengeme") + L(t + 3, "9.9.9.9", "/4?challengeme"), (t + 3) * S,
             W.RELOAD_RULES)]


def integration_rates(t):
    """banjax_integration_test.go:327-385 TestRegexesWithRates: hosts_to_skip
    on `.*`, 46 GETs within 60 s (httpStress sends repeat + 1) -> nginx_block,
    and the same burst from the global allow list."""
    L = W.standalone_line
    return [(L(t, "10.10.10.10", "/1"), t * S),
            (L(t + 2, "10.10.10.10", "/2"), (t + 2) * S),
            (L(t + 2, "11.11.11.11", "/45in60") * 46, (t + 2) * S),
            (L(t + 4, "11.11.11.11", "/45in60"), (t + 4) * S),
            (L(t + 4, "12.12.12.12", "/45in60-whitelist") * 46, (t + 4) * S),
            (L(t + 6, "12.12.12.12", "/45in60-whitelist"), (t + 6) * S)]


def main():
    t = 1700000000
    run("integration_challengeme", W.FIXTURE_RULES, integration_challengeme(t),
        "banjax_integration_test.go:293-325 + SIGHUP reload to fixtures/banjax-config-test-reload.yaml")
    run("integration_rates", W.REGEX_BANNER_RULES, integration_rates(t),
        "banjax_integration_test.go:327-385 with fixtures/banjax-config-test-regex-banner.yaml:63-92")
    run("consume_line_sequence", SEQ_CFG, seq_batches(),
        "regex_rate_limiter_test.go:77-260 TestConsumeLine, one batch per line")
    run("fixture_config", W.FIXTURE_RULES, [(fixture_lines(t), t * S), (fixture_lines(t + 1), (t + 1) * S)],
        "fixtures/banjax-config-test.yaml rules + allow lists; exemptions, per-site rule, OldLine, Error")
    run("edge_lines", EDGE_CFG, [(edge_lines(t), t * S), (edge_lines(t), (t + 1) * S)],
        "malformed headers, exotic ParseFloat tokens, net.ParseIP/CIDR edges, UTF-8, (?i) folding, \\b")
    run("tile_geometry", GEOM_CFG, [(geom_lines(t, 9, n=100), t * S)],
        "line lengths around the scan kernel's 4 KB tile / 512 B halo / 128 lines-per-tile limits")
    for wl, n, b, ips in [("cfg1", 3000, 2, 300), ("cfg2", 2000, 2, 200), ("cfg3", 3000, 2, 300),
                          ("cfg4", 40, 1, 10), ("cfg5", 3000, 2, 2500)]:
        y, batches = workload_batches(wl, n, b, ips)
        run("workload_" + wl, y, batches, "%s (BASELINE.json configs) scaled to %d lines, %d IPs" % (wl, n, ips))


if __name__ == "__main__":
    main()
