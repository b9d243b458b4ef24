"""A reload on another thread between a batch's process() and its Banner
replay must not pair the batch's trips with the new ruleset, nor
with the new decision lists / ban options: the reference swaps one
atomic config pointer and reads it once per line (config_holder.go:28,50-66,
regex_rate_limiter.go:59).  Here a batch holds the limiter's lock from
process() to its Banner replay; a reload publishes everything under it."""
import threading
import time
from types import SimpleNamespace

from banjax_amd import Config, MockBanner, RegexRateLimiter

OLD = """regexes_with_rates:
  - {rule: old-rule, regex: 'GET', interval: 1, hits_per_interval: 0, decision: iptables_block}
"""
NEW = """regexes_with_rates:
  - {rule: new-a, regex: 'POST', interval: 1, hits_per_interval: 0, decision: challenge}
  - {rule: new-b, regex: 'PUT', interval: 1, hits_per_interval: 0, decision: challenge}
"""


class ReloadingEngine:
    """Engine stand-in: process() returns one trip of rule 0 and, while the
    batch is in flight, another thread's reload lands."""

    def __init__(self):
        self.limiter = None
        self.pushed = []
        self.reloader = None

    def set_decision_lists(self, entries):
        self.pushed.append("lists")

    def set_ban_options(self, *a, **kw):
        self.pushed.append("options")

    def process(self, rs, data, now_ns, copy_results=False, emit_bans=False, **kw):
        n0 = len(self.pushed)
        self.reloader = threading.Thread(target=self.limiter.reload, args=(Config.from_yaml(NEW),))
        self.reloader.start()  # the concurrent reload
        time.sleep(0.3)
        # it waits for this batch: nothing of the new config reached the engine
        assert len(self.pushed) == n0 and self.limiter.ruleset.rules[0].rule == "old-rule"
        line = data.split(b"\n")[0]
        trip = SimpleNamespace(line_idx=0, line_offset=0, line_len=len(line), rule_idx=0, ts_ns=1700000000 * 10 ** 9,
                               ip_off=15, ip_len=7, host_off=27, host_len=5, rest_off=23, decision=4)
        res = SimpleNamespace(line_idx=0, rule_idx=0, skip_host=0, seen_ip=0, match_type=0, exceeded=1)
        return SimpleNamespace(trips=[trip], results=[res], line_flags=b"\x00", n_trips=1)


def test_batch_uses_one_config_snapshot():
    eng = ReloadingEngine()
    lim = RegexRateLimiter(Config.from_yaml(OLD), engine=eng, banner=MockBanner())
    eng.limiter = lim
    data = b"1700000000.000 1.2.3.4 GET a.com GET /x HTTP/1.1 ua\n"
    results, _ = lim.consume_lines(data, 1700000000 * 10 ** 9)
    eng.reloader.join(10)
    assert not eng.reloader.is_alive()
    assert [r.rule_name for r in results[0].rule_results] == ["old-rule"]
    d = lim.banner.decision_lists.expiring["1.2.3.4"]
    assert d.decision == 4  # the old rule's IptablesBlock, not the new rules' Challenge
    assert lim.ruleset.rules[0].rule == "new-a"  # the reload itself took effect
