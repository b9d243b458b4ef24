"""Host surface of the log tailer, mirroring reference internal/regex_rate_limiter.go.

The per-line work of consumeLine/applyRegexToLog runs on the MI355X
(bjx_process_batch); this module keeps the reference's types and side-effect
order: for every trip, in (line, rule) order, Banner.BanOrChallengeIp then
Banner.LogRegexBan (regex_rate_limiter.go:254-266), with the injected clock
`now_ns` standing in for time.Now().
"""
from __future__ import annotations

import datetime as _dt
import json
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from .config import ALLOW, CHALLENGE, IPTABLES_BLOCK, NGINX_BLOCK, Config, Ruleset, decision_string
from .engine import Engine

FIRST_TIME, OUTSIDE_INTERVAL, INSIDE_INTERVAL = 0, 1, 2
_MATCH_TYPE_NAMES = {FIRST_TIME: "FirstTime", OUTSIDE_INTERVAL: "OutsideInterval", INSIDE_INTERVAL: "InsideInterval"}
LINE_ERROR, LINE_OLD, LINE_EXEMPTED = 1, 2, 4


@dataclass
class RateLimitResult:
    """rate_limit.go:170-198."""
    match_type: int = FIRST_TIME
    exceeded: bool = False

    def to_json(self):
        return {"MatchType": _MATCH_TYPE_NAMES[self.match_type], "Exceeded": self.exceeded}


@dataclass
class RuleResult:
    """regex_rate_limiter.go:87-93."""
    rule_name: str
    regex_match: bool
    skip_host: bool
    seen_ip: bool
    rate_limit_result: RateLimitResult


@dataclass
class ConsumeLineResult:
    """regex_rate_limiter.go:80-85."""
    error: bool = False
    old_line: bool = False
    exempted: bool = False
    rule_results: List[RuleResult] = field(default_factory=list)


# ------------------------------------------------------------------ JSON

def _go_json_string(s: bytes) -> str:
    """encoding/json string encoding (escapeHTML on, Go >= 1.22 \\b/\\f forms,
    invalid UTF-8 -> \\ufffd, U+2028/2029 escaped)."""
    out = ['"']
    i, n = 0, len(s)
    while i < n:
        c = s[i]
        if c < 0x80:
            if c >= 0x20 and c not in (0x22, 0x5C, 0x3C, 0x3E, 0x26):
                out.append(chr(c))
            elif c == 0x5C:
                out.append("\\\\")
            elif c == 0x22:
                out.append('\\"')
            elif c == 0x08:
                out.append("\\b")
            elif c == 0x0C:
                out.append("\\f")
            elif c == 0x0A:
                out.append("\\n")
            elif c == 0x0D:
                out.append("\\r")
            elif c == 0x09:
                out.append("\\t")
            else:
                out.append("\\u00%02x" % c)
            i += 1
            continue
        r, w = _decode_rune(s, i)
        if r == 0xFFFD and w == 1:
            out.append("\\ufffd")
        elif r in (0x2028, 0x2029):
            out.append("\\u%04x" % r)
        else:
            out.append(s[i:i + w].decode("utf-8"))
        i += w
    out.append('"')
    return "".join(out)


def _decode_rune(s: bytes, i: int):
    """unicode/utf8.DecodeRune."""
    b0 = s[i]
    if b0 < 0x80:
        return b0, 1
    lo, hi = 0x80, 0xBF
    if 0xC2 <= b0 <= 0xDF:
        need, r = 1, b0 & 0x1F
    elif b0 == 0xE0:
        need, r, lo = 2, b0 & 0x0F, 0xA0
    elif 0xE1 <= b0 <= 0xEC or b0 in (0xEE, 0xEF):
        need, r = 2, b0 & 0x0F
    elif b0 == 0xED:
        need, r, hi = 2, b0 & 0x0F, 0x9F
    elif b0 == 0xF0:
        need, r, lo = 3, b0 & 0x07, 0x90
    elif 0xF1 <= b0 <= 0xF3:
        need, r = 3, b0 & 0x07
    elif b0 == 0xF4:
        need, r, hi = 3, b0 & 0x07, 0x8F
    else:
        return 0xFFFD, 1
    if i + need > len(s) - 1:
        return 0xFFFD, 1
    if not (lo <= s[i + 1] <= hi):
        return 0xFFFD, 1
    r = (r << 6) | (s[i + 1] & 0x3F)
    for k in range(2, need + 1):
        if not (0x80 <= s[i + k] <= 0xBF):
            return 0xFFFD, 1
        r = (r << 6) | (s[i + k] & 0x3F)
    return r, need + 1


_SPACES = {0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0, 0x1680, 0x2028, 0x2029, 0x202F, 0x205F, 0x3000}


def _is_space(r):
    return r in _SPACES or 0x2000 <= r <= 0x200A


def _trim_space(s: bytes) -> bytes:
    """strings.TrimSpace."""
    i = 0
    while i < len(s):
        r, w = _decode_rune(s, i)
        if not _is_space(r):
            break
        i += w
    s = s[i:]
    while s:
        start = len(s) - 1
        lim = 0
        while start > 0 and (s[start] & 0xC0) == 0x80 and lim < 3:
            start -= 1
            lim += 1
        r, w = _decode_rune(s, start)
        if w != len(s) - start:
            r, start = 0xFFFD, len(s) - 1
        if not _is_space(r):
            break
        s = s[:start]
    return s


class Zone:
    """The local time zone LogRegexBan formats its timestring in (logTime.Format
    in time.Local, iptables.go:187): a UTC offset before the first transition,
    then (UTC second, offset) changes in ascending order — the table
    bjx_ban_options carries to the device."""

    def __init__(self, offset_s: int = 0, transitions=()):
        self.offset_s = int(offset_s)
        self.transitions = [(int(a), int(o)) for a, o in transitions]
        self._at = [a for a, _ in self.transitions]

    @classmethod
    def fixed(cls, offset_s: int) -> "Zone":
        return cls(offset_s)

    @classmethod
    def from_tzinfo(cls, tz, first_year: int = 1970, last_year: int = 2100, start_s=None) -> "Zone":
        """Expand a tzinfo's offset changes over [first_year, last_year) (or from
        start_s): daily samples, each change pinned to the second by bisection.
        For a tzinfo without its TZif data; named zones use from_tzif."""
        def off(sec):
            return int(_dt.datetime.fromtimestamp(sec, tz).utcoffset().total_seconds())
        lo = int(_dt.datetime(first_year, 1, 1, tzinfo=_dt.timezone.utc).timestamp()) if start_s is None else int(start_s)
        hi = int(_dt.datetime(last_year, 1, 1, tzinfo=_dt.timezone.utc).timestamp())
        first = off(lo)
        trans, cur, t = [], first, lo
        while t < hi:
            nt = min(t + 86400, hi)
            o = off(nt)
            if o != cur:
                a, b = t, nt  # off(a) == cur, off(b) != cur
                while b - a > 1:
                    m = (a + b) // 2
                    if off(m) == cur:
                        a = m
                    else:
                        b = m
                cur = off(b)
                trans.append((b, cur))
                t = b
                continue
            t = nt
        return cls(first, trans)

    @classmethod
    def from_tzif(cls, data: bytes, tz_after=None, last_year: int = 2400) -> "Zone":
        """The zone as Go's time.LoadLocation reads a TZif file: every explicit
        transition of the 64-bit (v2+) data block, the offset before the first
        one chosen as Location.lookupFirstZone does (the first zone type if no
        transition uses it, else the first non-DST type), and after the last
        explicit transition the footer's rule, expanded (with tz_after, a tzinfo
        of the same zone; daily samples pinned by bisection) up to last_year."""
        import struct
        if data[:4] != b"TZif":
            raise ValueError("not a TZif file")
        ver = data[4]

        def counts(off):
            return struct.unpack(">6l", data[off + 20:off + 44])  # isut, isstd, leap, time, type, char
        isut, isstd, leap, timecnt, typecnt, charcnt = counts(0)
        base, tsize = 44, 4
        if ver >= ord("2"):
            off = 44 + timecnt * 5 + typecnt * 6 + charcnt + leap * 8 + isstd + isut
            isut, isstd, leap, timecnt, typecnt, charcnt = counts(off)
            base, tsize = off + 44, 8
        times = struct.unpack(">%d%s" % (timecnt, "q" if tsize == 8 else "l"), data[base:base + timecnt * tsize])
        p = base + timecnt * tsize
        idx = list(data[p:p + timecnt])
        p += timecnt
        types = [struct.unpack(">lBB", data[p + 6 * i:p + 6 * i + 6]) for i in range(typecnt)]  # utoff, isdst, desig
        first = 0
        if 0 in idx:  # time/zoneinfo.go lookupFirstZone, cases 2-4
            first = None
            if idx and types[idx[0]][1]:
                first = next((z for z in range(idx[0] - 1, -1, -1) if not types[z][1]), None)
            if first is None:
                first = next((z for z in range(typecnt) if not types[z][1]), 0)
        trans = [(int(t), int(types[i][0])) for t, i in zip(times, idx)]
        offset = int(types[first][0]) if types else 0
        if tz_after is not None:
            start = trans[-1][0] if trans else int(_dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc).timestamp())
            ext = cls.from_tzinfo(tz_after, last_year=last_year, start_s=start)
            trans += [(a, o) for a, o in ext.transitions if a > start]
        return cls(offset, trans)

    @classmethod
    def named(cls, name: str) -> "Zone":
        """An IANA zone from its TZif file (zoneinfo.TZPATH, else the tzdata package)."""
        import os
        import zoneinfo
        data = None
        for d in zoneinfo.TZPATH:
            f = os.path.join(d, name)
            if os.path.isfile(f):
                with open(f, "rb") as fh:
                    data = fh.read()
                break
        if data is None:
            import importlib.resources
            pkg, _, leaf = ("tzdata.zoneinfo/" + name).rpartition("/")
            data = importlib.resources.files(pkg.replace("/", ".")).joinpath(leaf).read_bytes()
        return cls.from_tzif(data, zoneinfo.ZoneInfo(name))

    def offset_at(self, sec: int) -> int:
        import bisect
        k = bisect.bisect_right(self._at, sec)
        return self.offset_s if k == 0 else self.transitions[k - 1][1]


def format_time(ns: int, zone=0) -> str:
    """logTime.Format("2006-01-02T15:04:05") in the local zone (a Zone, or a
    fixed offset in seconds east of UTC; UTC by default)."""
    sec = ns // 1_000_000_000
    sec += zone.offset_at(sec) if isinstance(zone, Zone) else int(zone)
    d = _dt.datetime(1970, 1, 1) + _dt.timedelta(seconds=sec)
    return "%04d-%02d-%02dT%02d:%02d:%02d" % (d.year, d.month, d.day, d.hour, d.minute, d.second)


# ------------------------------------------------------- decision lists

@dataclass
class ExpiringDecision:
    decision: int
    expires_ns: int
    ip: str
    from_baskerville: bool
    domain: str


class DynamicDecisionLists:
    """decision.go:377-439 (Update keeps only escalations)."""

    def __init__(self):
        self._mu = threading.Lock()
        self.expiring: Dict[str, ExpiringDecision] = {}

    def update(self, ip: str, expires_ns: int, decision: int, from_baskerville: bool, domain: str):
        with self._mu:
            old = self.expiring.get(ip)
            if old is not None and decision <= old.decision:
                return
            self.expiring[ip] = ExpiringDecision(decision, expires_ns, ip, from_baskerville, domain)

    def clear(self):
        """Clear (decision.go:540-546)."""
        with self._mu:
            self.expiring.clear()

    def check(self, ip: str, now_ns: int):
        """decision.go:474-500 (lazy delete on expiry)."""
        with self._mu:
            d = self.expiring.get(ip)
            if d is None:
                return None
            if now_ns - d.expires_ns > 0:
                del self.expiring[ip]
                return None
            return d


class Banner:
    """Banner.BanOrChallengeIp / LogRegexBan (iptables.go:179-228, 273-331)."""

    def __init__(self, decision_lists: DynamicDecisionLists):
        self.decision_lists = decision_lists
        self.ban_log: List[str] = []      # Logger lines
        self.ban_log_temp: List[str] = []  # LoggerTemp lines (disable_logging hosts)
        self.ipset: List[str] = []        # IPs an iptables ban would add (standalone: none)
        self.standalone = True
        self.zone = Zone()                # local zone of LogRegexBan's timestring

    def ban_or_challenge_ip(self, cfg: Config, ip: str, decision: int, domain: str, now_ns: int):
        expires = (now_ns + cfg.expiring_decision_ttl_seconds * 1_000_000_000) & ((1 << 64) - 1)
        if expires >= 1 << 63:
            expires -= 1 << 64
        self.decision_lists.update(ip, expires, decision, False, domain)
        if decision == IPTABLES_BLOCK and ip != "127.0.0.1" and not self.standalone:
            self.ipset.append(ip)

    def log_regex_ban(self, cfg: Config, log_time_ns: int, ip: bytes, rule_name: str, log_line: bytes, decision: int):
        words = log_line.split(b" ", 5)
        if len(words) < 6:
            return
        host = words[1].decode("utf-8", "surrogateescape")
        disable = 1 if cfg.disable_logging.get(host, False) else 0
        ua = _trim_space(words[5].split(b"|", 1)[0])
        parts = [
            '"path":' + _go_json_string(words[3]),
            '"timestring":' + _go_json_string(format_time(log_time_ns, self.zone).encode()),
            '"trigger":' + _go_json_string(rule_name.encode()),
            '"client_ua":' + _go_json_string(ua),
            '"client_ip":' + _go_json_string(ip),
            '"rule_type":"regex"',
            '"client_request_method":' + _go_json_string(words[0]),
            '"http_request_scheme":"https"',
            '"client_request_host":' + _go_json_string(words[1]),
            '"action":' + _go_json_string(decision_string(decision).encode()),
            '"number_of_fails":1',
            '"disable_logging":%d' % disable,
        ]
        line = "{" + ",".join(parts) + "}"
        (self.ban_log_temp if disable else self.ban_log).append(line)


    def apply_device_bans(self, cfg: Config, bans, trips, data):
        """The batch's device-emitted decision updates (one Update per tripped IP,
        same final lists as the per-trip BanOrChallengeIp replay) and ban-log lines."""
        for rec in bans.ips:
            t = trips[int(rec["trip_idx"])]
            line = bytes(data[t.line_offset:t.line_offset + t.line_len])
            ip = line[t.ip_off:t.ip_off + t.ip_len].decode("utf-8", "surrogateescape")
            host = line[t.host_off:t.host_off + t.host_len].decode("utf-8", "surrogateescape")
            self.decision_lists.update(ip, int(rec["expires_ns"]), int(rec["decision"]), False, host)
            if rec["iptables"] and ip != "127.0.0.1" and not self.standalone:
                self.ipset.append(ip)
        for kind, text in bans.lines():
            (self.ban_log_temp if kind == 2 else self.ban_log).append(text.decode("utf-8"))
        if trips:
            t = trips[-1]
            line = bytes(data[t.line_offset:t.line_offset + t.line_len])
            self.last_banned(line[t.ip_off:t.ip_off + t.ip_len].decode("utf-8", "surrogateescape"))

    def last_banned(self, ip: str):
        pass


class MockBanner(Banner):
    """regex_rate_limiter_test.go:27-75: records the last banned IP."""

    def __init__(self):
        super().__init__(DynamicDecisionLists())
        self.banned_ip = ""

    def ban_or_challenge_ip(self, cfg, ip, decision, domain, now_ns):
        self.banned_ip = ip
        super().ban_or_challenge_ip(cfg, ip, decision, domain, now_ns)

    def last_banned(self, ip: str):
        self.banned_ip = ip


# ------------------------------------------------------------ the tailer

class RegexRateLimitStates:
    """RegexRateLimitStates (rate_limit.go:17-103) backed by the engine's HBM tables."""

    def __init__(self, engine: Engine, names_fn):
        self._e = engine
        self._names = names_fn

    def get(self, ip: str) -> Optional[Dict[str, tuple]]:
        """Get(ip): copy of {rule name: (NumHits, IntervalStartTime ns)}, or None."""
        out = {}
        for name in self._names():
            st = self._e.state_get(ip, name)
            if st is not None:
                out[name] = st
        return out if out else None

    def __len__(self):
        return self._e.state_len()

    def __str__(self):
        return self._e.state_dump()


class _Snapshot:
    """One ConfigHolder value: a config and the ruleset compiled from it."""
    __slots__ = ("config", "ruleset")

    def __init__(self, config: Config, ruleset: Ruleset):
        self.config, self.ruleset = config, ruleset


class RegexRateLimiter:
    """Owns the config snapshot, its compiled ruleset and the engine; the
    equivalent of RunLogTailer's loop body over a batch of lines."""

    def __init__(self, cfg: Config, engine: Optional[Engine] = None, banner: Optional[Banner] = None,
                 device_bans: bool = False, tz_offset_s: int = 0, zone: Optional[Zone] = None,
                 device_ban_log: bool = True):
        """device_bans: the engine emits one decision update per tripped IP and
        the formatted ban-log lines (bjx_batch_bans) instead of
        the per-trip Banner replay on the host.  device_ban_log=False: the
        engine emits only the decision records (BJX_BAN_RECORDS_ONLY) and the
        host writes the LogRegexBan lines.  zone: time.Local of the ban log
        (default: the fixed offset tz_offset_s)."""
        self.engine = engine or Engine()
        self.banner = banner or MockBanner()
        self.device_bans = device_bans
        self.device_ban_log = device_ban_log
        # one batch at a time sees one (config, ruleset, decision lists, ban
        # options): reload() publishes all of them under this lock
        self._mu = threading.Lock()
        self.zone = zone if zone is not None else Zone.fixed(tz_offset_s)
        self.banner.zone = self.zone
        self._seen_names: Dict[str, None] = {}
        self.states = RegexRateLimitStates(self.engine, lambda: list(self._seen_names))
        self.reload(cfg)

    def reload(self, cfg: Config):
        """ConfigHolder.Reload (config_holder.go:55-66): compile first; keep the old
        ruleset if the new config does not compile; state survives (keyed by name).
        The (config, ruleset) pair is published as one object, like the
        reference's atomic config pointer (config_holder.go:28,63): a batch
        takes one snapshot and uses it from process() to its Banner replay, so a
        reload on another thread takes effect at the next batch."""
        rs = Ruleset(cfg)  # compiled outside the lock: a bad config raises here, nothing changes
        with self._mu:
            for r in rs.rules:
                self._seen_names.setdefault(r.rule, None)
            # the engine's decision lists and ban options first, then the
            # snapshot: no batch runs between them (it holds the same lock)
            self.engine.set_decision_lists(cfg.decision_entries)
            self.engine.set_ban_options(cfg.expiring_decision_ttl_seconds,
                                        [h for h, v in cfg.disable_logging.items() if v], zone=self.zone)
            self._snap = _Snapshot(cfg, rs)

    def sighup(self, cfg: Config):
        """The reference's SIGHUP handler (banjax.go:101-115): Reload; on
        success the static lists follow the new config (pushed by reload) and
        the dynamic decision lists are cleared.  A config that does not compile
        raises and changes nothing, as `continue` does there."""
        self.reload(cfg)
        with self._mu:
            self.banner.decision_lists.clear()

    @property
    def config(self) -> Config:
        return self._snap.config

    @property
    def ruleset(self) -> Ruleset:
        return self._snap.ruleset

    def consume_lines(self, data: bytes, now_ns: int, want_results: bool = True):
        """consumeLine for every complete line; returns (results, batch output)."""
        with self._mu:
            snap = self._snap
            out = self.engine.process(snap.ruleset, data, now_ns, copy_results=want_results, **self._ban_kw())
            return self._finish(snap, data, out, now_ns, want_results)

    def _ban_kw(self):
        if not self.device_bans:
            return {}
        return {"emit_bans": True} if self.device_ban_log else {"emit_bans": True, "ban_log": False}

    def consume_device_batch(self, host_view, device_ptr: Optional[int], nbytes: int, now_ns: int,
                             want_results: bool = True):
        """consumeLine over a batch already in HBM (the tailer's copy); host_view
        holds the same bytes for the Banner's log lines.  device_ptr None: host."""
        with self._mu:
            snap = self._snap
            if device_ptr is None:
                out = self.engine.process(snap.ruleset, bytes(host_view[:nbytes]), now_ns, copy_results=want_results,
                                          **self._ban_kw())
            else:
                out = self.engine.process(snap.ruleset, None, now_ns, copy_results=want_results, device_ptr=device_ptr,
                                          nbytes=nbytes, **self._ban_kw())
            return self._finish(snap, host_view, out, now_ns, want_results)

    def _finish(self, snap, data, out, now_ns: int, want_results: bool):
        """Banner replay of the trips in reference order (regex_rate_limiter.go:254-266)
        and, if asked, the ConsumeLineResults, against the batch's snapshot."""
        rules = snap.ruleset.rules
        if self.device_bans:
            self.banner.apply_device_bans(snap.config, self.engine.bans(), out.trips, data)
            if not self.device_ban_log:  # records only: LogRegexBan per trip on the host, in order
                rules, config = snap.ruleset.rules, snap.config
                for t in out.trips:
                    line = bytes(data[t.line_offset:t.line_offset + t.line_len])
                    rule = rules[t.rule_idx]
                    self.banner.log_regex_ban(config, t.ts_ns, line[t.ip_off:t.ip_off + t.ip_len], rule.rule,
                                              line[t.rest_off:], rule.decision)
        else:
            self._replay_trips(snap, data, out, now_ns)
        if not want_results:
            return None, out
        results = [ConsumeLineResult(error=bool(f & LINE_ERROR), old_line=bool(f & LINE_OLD),
                                     exempted=bool(f & LINE_EXEMPTED)) for f in out.line_flags]
        for r in out.results:
            results[r.line_idx].rule_results.append(RuleResult(
                rule_name=rules[r.rule_idx].rule, regex_match=True, skip_host=bool(r.skip_host),
                seen_ip=bool(r.seen_ip), rate_limit_result=RateLimitResult(r.match_type, bool(r.exceeded))))
        return results, out

    def _replay_trips(self, snap, data, out, now_ns: int):
        rules, config = snap.ruleset.rules, snap.config
        for t in out.trips:
            line = bytes(data[t.line_offset:t.line_offset + t.line_len])
            ip = line[t.ip_off:t.ip_off + t.ip_len]
            host = line[t.host_off:t.host_off + t.host_len]
            rest = line[t.rest_off:]
            rule = rules[t.rule_idx]
            self.banner.ban_or_challenge_ip(config, ip.decode("utf-8", "surrogateescape"), rule.decision,
                                            host.decode("utf-8", "surrogateescape"), now_ns)
            self.banner.log_regex_ban(config, t.ts_ns, ip, rule.rule, rest, rule.decision)


def consume_line(limiter: RegexRateLimiter, text: str, now_ns: int) -> ConsumeLineResult:
    """consumeLine(line, ...) for one tail.Line (its Text has no trailing '\\n')."""
    res, _ = limiter.consume_lines(text.encode("utf-8", "surrogateescape") + b"\n", now_ns)
    return res[0]


def result_to_json(r: ConsumeLineResult) -> str:
    """json.MarshalIndent(result) as printed by RunLogTailer in debug mode (:68-75)."""
    return json.dumps({"Error": r.error, "OldLine": r.old_line, "Exempted": r.exempted,
                       "RuleResults": None if not r.rule_results else [
                           {"RuleName": x.rule_name, "RegexMatch": x.regex_match, "SkipHost": x.skip_host,
                            "SeenIp": x.seen_ip, "RateLimitResult": x.rate_limit_result.to_json()}
                           for x in r.rule_results]}, indent=2)
