"""Config reload through the GPU engine: ConfigHolder.Reload
(internal/config_holder.go:55-66) swaps the compiled ruleset while
RegexRateLimitStates persists, keyed by (ip, rule *name*)
(internal/rate_limit.go:37-78; state survives reload, banjax.go:113-115).
Rules that keep their name keep counting with the new interval / limit /
decision; renamed rules start fresh; removed names keep their old state; a
config that fails to compile leaves the previous ruleset in force
(config.go:110-113).  Bit-exact against the oracle fed the same configs.
"""
import pytest

import workloads as W
from banjax_amd import Config
from banjax_amd.config import ConfigError
from tests.parity import Pair, oracle_config

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from banjax_amd import Engine
    e = Engine()
    yield e
    e.close()


RELOAD_B = W.DDOS_RULES.replace('''  - rule: "burst2"
    regex: '^(GET|POST) \\S+ (GET|POST) \\/(api|search)'
    interval: 5
    hits_per_interval: 2
    decision: challenge''', '''  - rule: "burst2"
    regex: 'POST'
    interval: 2
    hits_per_interval: 1
    decision: nginx_block
  - rule: "instant"
    regex: 'search'
    interval: 3
    hits_per_interval: 4
    decision: iptables_block''').replace('rule: "flood10"', 'rule: "flood10-renamed"') + '''per_site_regexes_with_rates:
  "site001.example.com":
    - rule: "site burst"
      regex: 'GET'
      interval: 1
      hits_per_interval: 3
      decision: challenge
expiring_decision_ttl_seconds: 30
'''


def _reload(pair, yaml_text):
    cfg = Config.from_yaml(yaml_text)
    pair.lim.reload(cfg)
    pair.cfg, pair.ocfg, pair.n_rules = cfg, oracle_config(cfg), len(cfg.all_rules())


def test_reload_keeps_state_by_rule_name(engine):
    assert RELOAD_B != W.DDOS_RULES and "flood10-renamed" in RELOAD_B
    w = W.scaled(W.CFG5, 80_000, n_ips=1_500)
    per = 20_000
    pair = Pair(w.rules_yaml, engine, device_bans=True)
    ips = set()
    for b, text in enumerate([None, RELOAD_B, None, RELOAD_B]):
        if text is not None:
            _reload(pair, text)
        elif b:
            _reload(pair, w.rules_yaml)
        data = w.host_lines(b * per, per)
        for ln in data.split(b"\n")[:200]:
            parts = ln.split(b" ")
            if len(parts) > 2:
                ips.add(parts[1].decode())
        pair.feed(data, w.now_ns(b * per, per))
    names = {"instant", "burst2", "flood10", "flood10-renamed", "site burst"}
    ost, eng = pair.ost, pair.engine
    assert eng.state_len() == len(ost)
    for ip in sorted(ips)[:80]:
        for n in names:
            assert eng.state_get(ip, n) == ost.get(ip, n), (ip, n)
    pair.compare_state()


def test_reload_with_bad_regex_keeps_previous_ruleset(engine):
    w = W.scaled(W.CFG5, 10_000, n_ips=500)
    pair = Pair(w.rules_yaml, engine)
    pair.feed(w.host_lines(0, 5_000), w.now_ns(0, 5_000))
    bad = w.rules_yaml.replace("'.*'", "'(?invalid'")
    with pytest.raises(ConfigError):
        pair.lim.reload(Config.from_yaml(bad))
    pair.feed(w.host_lines(5_000, 5_000), w.now_ns(5_000, 5_000))  # old ruleset still in force
    pair.compare_state()
