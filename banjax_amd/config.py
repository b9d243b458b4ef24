"""The regexes_with_rates config schema (reference internal/config.go).

Mirrors the YAML surface the Go host keeps: `regexes_with_rates`,
`per_site_regexes_with_rates`, `global_decision_lists`,
`per_site_decision_lists`, `expiring_decision_ttl_seconds`,
`disable_logging`.  Rule compilation (regexp.Compile, config.go:110) happens
in the HIP library (bjx_ruleset_compile); a compile error fails the load, as
`RegexWithRate.UnmarshalYAML` does (config.go:110-113).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import yaml

from . import _lib

# Decision, reference internal/decision.go:20-58
ALLOW, CHALLENGE, NGINX_BLOCK, IPTABLES_BLOCK = 1, 2, 3, 4
_DECISIONS = {"allow": ALLOW, "challenge": CHALLENGE, "nginx_block": NGINX_BLOCK, "iptables_block": IPTABLES_BLOCK}
_DECISION_NAMES = {ALLOW: "Allow", CHALLENGE: "Challenge", NGINX_BLOCK: "NginxBlock", IPTABLES_BLOCK: "IptablesBlock"}


class ConfigError(ValueError):
    pass


def parse_decision(s: str) -> int:
    """ParseDecision, decision.go:30-43."""
    try:
        return _DECISIONS[s]
    except KeyError:
        raise ConfigError("invalid decision: %s" % (s,))


def decision_string(d: int) -> str:
    """Decision.String, decision.go:45-58."""
    return _DECISION_NAMES.get(d, "")


def interval_ns(seconds) -> int:
    """time.Duration(i.Interval * float64(time.Second.Nanoseconds())), config.go:116
    (float64 multiply, then int64 conversion with amd64 out-of-range semantics)."""
    x = float(seconds) * 1e9
    if not (-9223372036854775808.0 <= x < 9223372036854775808.0):
        return -(1 << 63)
    return int(x)


@dataclass
class RegexWithRate:
    """config.go:87-94."""
    rule: str
    regex: str
    interval: int               # ns
    hits_per_interval: int
    decision: int
    hosts_to_skip: Dict[str, bool] = field(default_factory=dict)

    @classmethod
    def from_yaml(cls, m) -> "RegexWithRate":
        """RegexWithRate.UnmarshalYAML, config.go:96-131 (compilation is deferred to the ruleset)."""
        if not isinstance(m, dict):
            raise ConfigError("regex rule must be a mapping")
        hits = m.get("hits_per_interval", 0)
        if isinstance(hits, bool) or not isinstance(hits, int):
            raise ConfigError("hits_per_interval must be an int")
        skip = m.get("hosts_to_skip") or {}
        return cls(rule="" if m.get("rule") is None else str(m.get("rule")),
                   regex="" if m.get("regex") is None else str(m.get("regex")),
                   interval=interval_ns(m.get("interval", 0) or 0),
                   hits_per_interval=int(hits),
                   decision=parse_decision(m.get("decision", "")),
                   hosts_to_skip={str(k): bool(v) for k, v in skip.items()})


@dataclass
class Config:
    regexes_with_rates: List[RegexWithRate] = field(default_factory=list)
    per_site_regexes_with_rates: Dict[str, List[RegexWithRate]] = field(default_factory=dict)
    # (site or None, decision, ip) in document order
    decision_entries: List[Tuple[Optional[str], int, str]] = field(default_factory=list)
    expiring_decision_ttl_seconds: int = 0
    disable_logging: Dict[str, bool] = field(default_factory=dict)
    debug: bool = False

    @classmethod
    def from_yaml(cls, text: str) -> "Config":
        doc = yaml.safe_load(text) or {}
        c = cls()
        c.regexes_with_rates = [RegexWithRate.from_yaml(r) for r in (doc.get("regexes_with_rates") or [])]
        for host, rules in (doc.get("per_site_regexes_with_rates") or {}).items():
            c.per_site_regexes_with_rates[str(host)] = [RegexWithRate.from_yaml(r) for r in (rules or [])]
        for dec, ips in (doc.get("global_decision_lists") or {}).items():
            d = parse_decision(dec)
            for ip in ips or []:
                c.decision_entries.append((None, d, str(ip)))
        for site, lists in (doc.get("per_site_decision_lists") or {}).items():
            for dec, ips in (lists or {}).items():
                d = parse_decision(dec)
                for ip in ips or []:
                    c.decision_entries.append((str(site), d, str(ip)))
        c.expiring_decision_ttl_seconds = int(doc.get("expiring_decision_ttl_seconds") or 0)
        c.disable_logging = {str(k): bool(v) for k, v in (doc.get("disable_logging") or {}).items()}
        c.debug = bool(doc.get("debug", False))
        return c

    def all_rules(self) -> List[RegexWithRate]:
        """Ruleset index order: global rules, then each site's rules."""
        out = list(self.regexes_with_rates)
        for host in self.per_site_regexes_with_rates:
            out.extend(self.per_site_regexes_with_rates[host])
        return out


class Ruleset:
    """An immutable compiled ruleset (bjx_ruleset_compile).  A reload compiles a
    new one; the engine keeps rate-limit state keyed by rule name."""

    def __init__(self, cfg: Config):
        L = _lib.lib()
        self._keep = []
        self.rules = cfg.all_rules()

        def spec(r: RegexWithRate) -> _lib.RuleSpec:
            skips = [h for h, v in r.hosts_to_skip.items() if v]
            arr = (_lib.Str * max(1, len(skips)))(*[_lib.mkstr(h) for h in skips])
            self._keep.append(arr)
            s = _lib.RuleSpec(_lib.mkstr(r.rule), _lib.mkstr(r.regex), r.interval, r.hits_per_interval, r.decision,
                              C.cast(arr, C.POINTER(_lib.Str)), len(skips))
            self._keep.append(s)
            return s

        g = (_lib.RuleSpec * max(1, len(cfg.regexes_with_rates)))(*[spec(r) for r in cfg.regexes_with_rates])
        sites = []
        for host, rules in cfg.per_site_regexes_with_rates.items():
            arr = (_lib.RuleSpec * max(1, len(rules)))(*[spec(r) for r in rules])
            self._keep.append(arr)
            sites.append(_lib.SiteRules(_lib.mkstr(host), C.cast(arr, C.POINTER(_lib.RuleSpec)), len(rules)))
        sarr = (_lib.SiteRules * max(1, len(sites)))(*sites)
        h = C.c_void_p()
        err_rule = C.c_int64(-1)
        err = C.create_string_buffer(1024)
        rc = L.bjx_ruleset_compile(g, len(cfg.regexes_with_rates), sarr, len(sites), C.byref(h), C.byref(err_rule),
                                   err, 1024)
        self._keep = None
        if rc != _lib.OK:
            raise ConfigError(err.value.decode(errors="replace"))
        self._h = h

    @property
    def handle(self):
        return self._h

    def __len__(self):
        return _lib.lib().bjx_ruleset_num_rules(self._h)

    def rule_info(self, i):
        st, cl, fl = C.c_uint32(), C.c_uint32(), C.c_uint32()
        _lib.lib().bjx_ruleset_rule_info(self._h, i, C.byref(st), C.byref(cl), C.byref(fl))
        return st.value, cl.value, fl.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib._lib is not None:
            _lib._lib.bjx_ruleset_release(h)
