"""ORACLE — test infrastructure only.

ctypes wrapper around oracle/build/libbjx_oracle.so, the plain-C restatement of
banjax's regex rate-limiting log tailer (see bjx_oracle.c for the reference
file:line of every function).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg import this module; the product (banjax_amd/)
never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libbjx_oracle.so")

ALLOW, CHALLENGE, NGINX_BLOCK, IPTABLES_BLOCK = 1, 2, 3, 4
DECISIONS = {"allow": ALLOW, "challenge": CHALLENGE, "nginx_block": NGINX_BLOCK,
             "iptables_block": IPTABLES_BLOCK}
LINE_ERROR, LINE_OLD, LINE_EXEMPTED = 1, 2, 4


class RuleResult(C.Structure):
    _fields_ = [("line_idx", C.c_uint64), ("rule_id", C.c_uint32), ("rule_pos", C.c_uint16),
                ("skip_host", C.c_uint8), ("seen_ip", C.c_uint8), ("match_type", C.c_uint8),
                ("exceeded", C.c_uint8), ("_pad", C.c_uint8 * 2)]


def build() -> str:
    """Compile the oracle with its own Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, sz, i64, u8p = C.c_void_p, C.c_size_t, C.c_int64, C.POINTER(C.c_uint8)
        L.gre_compile.restype = vp
        L.gre_compile.argtypes = [C.c_char_p, sz, C.c_char_p, sz]
        L.gre_parse_check.restype = C.c_int
        L.gre_parse_check.argtypes = [C.c_char_p, sz, C.c_char_p, sz]
        L.gre_match.restype = C.c_int
        L.gre_match.argtypes = [vp, C.c_char_p, sz]
        L.gre_free.argtypes = [vp]
        L.orc_cfg_new.restype = vp
        L.orc_cfg_free.argtypes = [vp]
        L.orc_cfg_add_rule.restype = C.c_int
        L.orc_cfg_add_rule.argtypes = [vp, C.c_char_p, sz, C.c_char_p, sz, C.c_char_p, sz, i64, i64,
                                       C.c_int, C.c_char_p, sz]
        L.orc_cfg_add_skip_host.argtypes = [vp, C.c_int, C.c_char_p, sz]
        L.orc_cfg_add_decision_ip.argtypes = [vp, C.c_char_p, sz, C.c_int, C.c_char_p, sz]
        L.orc_cfg_set_expiring_ttl.argtypes = [vp, i64]
        L.orc_cfg_add_disable_logging.argtypes = [vp, C.c_char_p, sz]
        L.orc_state_new.restype = vp
        L.orc_state_free.argtypes = [vp]
        L.orc_consume_batch.restype = i64
        L.orc_consume_batch.argtypes = [vp, vp, C.c_char_p, sz, i64, u8p, C.POINTER(RuleResult), sz,
                                        C.POINTER(sz), C.POINTER(sz)]
        L.orc_state_get.restype = C.c_int
        L.orc_state_get.argtypes = [vp, C.c_char_p, sz, C.c_char_p, sz, C.POINTER(i64), C.POINTER(i64)]
        L.orc_state_len.restype = i64
        L.orc_state_len.argtypes = [vp]
        L.orc_decision_get.restype = C.c_int
        L.orc_decision_get.argtypes = [vp, C.c_char_p, sz, C.POINTER(C.c_int), C.POINTER(i64), C.c_char_p, sz]
        L.orc_decision_len.restype = i64
        L.orc_decision_len.argtypes = [vp]
        L.orc_decision_clear.restype = None
        L.orc_decision_clear.argtypes = [vp]
        L.orc_last_banned_ip.restype = sz
        L.orc_last_banned_ip.argtypes = [vp, C.c_char_p, sz]
        L.orc_ban_log.restype = sz
        L.orc_ban_log.argtypes = [vp, C.c_char_p, sz]
        L.orc_parse_float.restype = C.c_int
        L.orc_parse_float.argtypes = [C.c_char_p, sz, C.POINTER(C.c_double)]
        L.orc_parse_ip.restype = C.c_int
        L.orc_parse_ip.argtypes = [C.c_char_p, sz, C.c_uint8 * 16]
        _lib = L
    return _lib


def _b(x) -> bytes:
    return x if isinstance(x, bytes) else x.encode()


class Regex:
    """regexp.Compile / (*Regexp).Match restated (go_regexp.c)."""

    def __init__(self, pattern):
        p = _b(pattern)
        err = C.create_string_buffer(512)
        self._h = lib().gre_compile(p, len(p), err, 512)
        if not self._h:
            raise ValueError(err.value.decode(errors="replace"))

    def match(self, text) -> bool:
        t = _b(text)
        return bool(lib().gre_match(self._h, t, len(t)))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.gre_free(self._h)


def compile_error(pattern):
    """None if pattern compiles, else the Go-style error string."""
    try:
        Regex(pattern)
        return None
    except ValueError as e:
        return str(e)


def parse_float(s):
    out = C.c_double()
    b = _b(s)
    rc = lib().orc_parse_float(b, len(b), C.byref(out))
    return rc, out.value


def parse_ip(s):
    out = (C.c_uint8 * 16)()
    b = _b(s)
    ok = lib().orc_parse_ip(b, len(b), out)
    return bytes(out) if ok else None


class Config:
    """Rules + static decision lists, mirroring config.go / decision.go."""

    def __init__(self, expiring_ttl_s: int = 10):
        self._h = lib().orc_cfg_new()
        lib().orc_cfg_set_expiring_ttl(self._h, expiring_ttl_s)
        self.rule_names = []

    def add_rule(self, name, regex, interval_ns, hits, decision, site=None, hosts_to_skip=()):
        err = C.create_string_buffer(512)
        n, r = _b(name), _b(regex)
        s = _b(site) if site is not None else None
        rid = lib().orc_cfg_add_rule(self._h, s, len(s) if s else 0, n, len(n), r, len(r),
                                     int(interval_ns), int(hits), int(decision), err, 512)
        if rid < 0:
            raise ValueError(err.value.decode(errors="replace"))
        for h in hosts_to_skip:
            hb = _b(h)
            lib().orc_cfg_add_skip_host(self._h, rid, hb, len(hb))
        self.rule_names.append(name)
        return rid

    def add_decision_ip(self, decision, ip, site=None):
        s = _b(site) if site is not None else None
        ib = _b(ip)
        lib().orc_cfg_add_decision_ip(self._h, s, len(s) if s else 0, int(decision), ib, len(ib))

    def add_disable_logging(self, host):
        hb = _b(host)
        lib().orc_cfg_add_disable_logging(self._h, hb, len(hb))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orc_cfg_free(self._h)


class State:
    """RegexRateLimitStates + DynamicDecisionLists + MockBanner/ban log."""

    def __init__(self):
        self._h = lib().orc_state_new()

    def consume(self, cfg: Config, buf: bytes, now_ns: int, cap=None):
        """Run consumeLine over every complete line; returns (flags, results, consumed)."""
        buf = _b(buf)
        n_lines = buf.count(b"\n")
        flags = (C.c_uint8 * max(n_lines, 1))()
        cap = cap if cap is not None else max(16, n_lines * 4)
        res = (RuleResult * cap)()
        nres, consumed = C.c_size_t(), C.c_size_t()
        lib().orc_consume_batch(cfg._h, self._h, buf, len(buf), int(now_ns),
                                C.cast(flags, C.POINTER(C.c_uint8)), res, cap,
                                C.byref(nres), C.byref(consumed))
        if nres.value > cap:
            raise RuntimeError("result capacity too small")
        return list(flags[:n_lines]), [res[i] for i in range(nres.value)], consumed.value

    def get(self, ip, name):
        h, s = C.c_int64(), C.c_int64()
        ib, nb = _b(ip), _b(name)
        if lib().orc_state_get(self._h, ib, len(ib), nb, len(nb), C.byref(h), C.byref(s)):
            return h.value, s.value
        return None

    def __len__(self):
        return lib().orc_state_len(self._h)

    def decision(self, ip):
        d, e = C.c_int(), C.c_int64()
        ib = _b(ip)
        cap = 512
        while True:
            dom = C.create_string_buffer(cap)
            r = lib().orc_decision_get(self._h, ib, len(ib), C.byref(d), C.byref(e), dom, cap)
            if r == 0:
                return None
            if r <= cap:
                return d.value, e.value, dom.raw[:r - 1].decode(errors="replace")
            cap = r

    def decisions_len(self):
        return lib().orc_decision_len(self._h)

    def decisions_clear(self):
        """DynamicDecisionLists.Clear (decision.go:540-546), as banjax.go:101-115 after a reload."""
        lib().orc_decision_clear(self._h)

    def banned_ip(self):
        n = lib().orc_last_banned_ip(self._h, None, 0)
        buf = C.create_string_buffer(n + 1)
        lib().orc_last_banned_ip(self._h, buf, n + 1)
        return buf.raw[:n].decode(errors="replace")

    def ban_log(self):
        n = lib().orc_ban_log(self._h, None, 0)
        buf = C.create_string_buffer(n + 1)
        lib().orc_ban_log(self._h, buf, n)
        return buf.raw[:n].decode(errors="replace")

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orc_state_free(self._h)
