"""Parity harness: run the same config + log bytes through the oracle (CPU
restatement, test infrastructure) and the MI355X engine (product), and compare
everything consumeLine produces: per-line Error/OldLine/Exempted, the
RuleResults in reference order, the rate-limit trips, the final
RegexRateLimitStates, and the decisions/ban-log lines the Banner replay makes.
"""
from __future__ import annotations

from oracle import oracle as O

from banjax_amd import Config, Engine, MockBanner, RegexRateLimiter


def oracle_config(cfg: Config) -> O.Config:
    oc = O.Config(expiring_ttl_s=cfg.expiring_decision_ttl_seconds)
    for r in cfg.regexes_with_rates:
        oc.add_rule(r.rule, r.regex, r.interval, r.hits_per_interval, r.decision,
                    hosts_to_skip=[h for h, v in r.hosts_to_skip.items() if v])
    for host, rules in cfg.per_site_regexes_with_rates.items():
        for r in rules:
            oc.add_rule(r.rule, r.regex, r.interval, r.hits_per_interval, r.decision, site=host,
                        hosts_to_skip=[h for h, v in r.hosts_to_skip.items() if v])
    for site, dec, ip in cfg.decision_entries:
        oc.add_decision_ip(dec, ip, site=site)
    for h, v in cfg.disable_logging.items():
        if v:
            oc.add_disable_logging(h)
    return oc


class Pair:
    """An oracle and an engine fed identical batches."""

    def __init__(self, cfg_yaml: str, engine: Engine = None, device_bans: bool = False):
        self.cfg = Config.from_yaml(cfg_yaml)
        self.ocfg = oracle_config(self.cfg)
        self.ost = O.State()
        self.engine = engine or Engine()
        self.engine.state_clear()
        self.lim = RegexRateLimiter(self.cfg, engine=self.engine, banner=MockBanner(), device_bans=device_bans)
        self.n_rules = len(self.cfg.all_rules())

    def feed(self, data: bytes, now_ns: int, check=True, want_results=True):
        """want_results=False: the engine's trip-only path (no RuleResult copies,
        the bench's); the states, decisions and ban log compared by
        compare_state still check every trip and its order."""
        before = self.engine.state_len()
        oflags, ores, oconsumed = self.ost.consume(self.ocfg, data, now_ns,
                                                   cap=(data.count(b"\n") + 1) * (self.n_rules + 1))
        results, out = self.lim.consume_lines(data, now_ns, want_results=want_results)
        if not want_results:
            assert out.consumed_bytes == oconsumed
            assert out.n_trips == sum(1 for r in ores if r.exceeded)
            return out
        if check:
            try:
                compare_batch(oflags, ores, oconsumed, out)
            except AssertionError:
                self._explain(data, ores, out, before)
                raise
        return out

    def _explain(self, data, ores, out, states_before):
        """Diagnostics for a rate-limit outcome mismatch: every result of the
        first differing (ip, rule) in this batch, both sides, and both states."""
        lines = data.split(b"\n")
        names = [r.rule for r in self.cfg.all_rules()]
        for k, (g, o) in enumerate(zip(out.results, ores)):
            if (g.match_type, g.exceeded) == (o.match_type, o.exceeded):
                continue
            ip = lines[g.line_idx].split(b" ")[1].decode(errors="replace")
            name = names[g.rule_idx]
            seq = [(i, r.line_idx, r.match_type, r.exceeded, ores[i].match_type, ores[i].exceeded)
                   for i, r in enumerate(out.results) if i < len(ores) and names[r.rule_idx] == name
                   and lines[r.line_idx].split(b" ")[1].decode(errors="replace") == ip]
            print("MISMATCH result %d ip=%s rule=%s states before batch gpu=%d; (idx, line, gpu mt, ex, oracle mt, ex): %s"
                  % (k, ip, name, states_before, seq[:12]), flush=True)
            print("  gpu state", self.engine.state_get(ip, name), "oracle state", self.ost.get(ip, name),
                  "gpu len", self.engine.state_len(), "oracle len", len(self.ost), "stats", self.engine.scan_stats(), flush=True)
            break

    def compare_state(self, ips=None):
        """Final RegexRateLimitStates for every (ip, rule name), Len(), and the
        decision list the Banner replay built."""
        names = sorted(set(r.rule for r in self.cfg.all_rules()))
        assert self.engine.state_len() == len(self.ost), (self.engine.state_len(), len(self.ost))
        for ip in ips or []:
            for n in names:
                g, o = self.engine.state_get(ip, n), self.ost.get(ip, n)
                assert g == o, (ip, n, g, o)
        dl = self.lim.banner.decision_lists.expiring
        assert len(dl) == self.ost.decisions_len()
        for ip, d in dl.items():
            od = self.ost.decision(ip)
            assert od is not None and od[0] == d.decision and od[1] == d.expires_ns and od[2] == d.domain, (ip, od, d)
        if self.ost.banned_ip() or self.lim.banner.banned_ip:
            assert self.lim.banner.banned_ip == self.ost.banned_ip()
        # ban log (LogRegexBan JSON), in order
        olog = [l for l in self.ost.ban_log().split("\n") if l]
        glog = ["0 " + l for l in self.lim.banner.ban_log] + ["1 " + l for l in self.lim.banner.ban_log_temp]
        if not self.lim.banner.ban_log_temp:
            assert olog == glog
        else:
            assert sorted(olog) == sorted(glog)


def compare_batch(oflags, ores, oconsumed, out):
    assert out.consumed_bytes == oconsumed
    assert out.n_lines == len(oflags)
    gflags = list(out.line_flags)
    if gflags != oflags:
        bad = [i for i in range(len(oflags)) if gflags[i] != oflags[i]][:10]
        raise AssertionError("line flags differ at %s: gpu=%s oracle=%s" %
                             (bad, [gflags[i] for i in bad], [oflags[i] for i in bad]))
    for k, (g, o) in enumerate(zip(out.results, ores)):
        gt = (g.line_idx, g.rule_idx, g.rule_pos, g.skip_host, g.seen_ip, g.match_type, g.exceeded)
        ot = (o.line_idx, o.rule_id, o.rule_pos, o.skip_host, o.seen_ip, o.match_type, o.exceeded)
        if gt != ot:
            raise AssertionError("RuleResult %d differs: gpu=%s oracle=%s" % (k, gt, ot))
    assert out.n_results == len(ores), (out.n_results, len(ores))
    trips = [(o.line_idx, o.rule_id) for o in ores if o.exceeded]
    assert [(t.line_idx, t.rule_idx) for t in out.trips] == trips
