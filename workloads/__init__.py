"""Benchmark / test workloads (BASELINE.json `configs`), synthetic and seeded.

Not product code.  Lines come from workloads/synth.hip (host and device
renderings of the same pure function of (cfg, line index)); rule sets are YAML
in the reference's `regexes_with_rates` schema.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, replace

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "libbjx_synth.so")
T0_MS = 1_700_000_000_000


class SynthCfg(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("first_line", C.c_uint64), ("n_lines", C.c_uint64), ("t0_ms", C.c_int64),
                ("us_per_line", C.c_uint32), ("n_ips", C.c_uint32), ("n_hosts", C.c_uint32),
                ("other_host_pct", C.c_uint32), ("trigger_permille", C.c_uint32), ("ua_heavy", C.c_uint32),
                ("ipv6_pct", C.c_uint32), ("ts_decimals", C.c_uint32), ("fixture_hosts", C.c_uint32),
                ("ip_mode", C.c_uint32), ("zipf_milli", C.c_uint32), ("hot_pct", C.c_uint32), ("_pad", C.c_uint32)]

IP_UNIFORM, IP_ZIPF, IP_DISTINCT = 0, 1, 2


HOST_APPLY_LIB = os.path.join(HERE, "lib", "libbjx_host_apply.so")


def build(force=False):
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    src = os.path.join(HERE, "synth.hip")
    if force or not os.path.exists(LIB) or os.path.getmtime(src) > os.path.getmtime(LIB):
        subprocess.run(["hipcc", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "--offload-arch=%s" % os.environ.get("BJX_OFFLOAD_ARCH", "gfx950"),
                        "-o", LIB, src], check=True)
    ha = os.path.join(HERE, "host_apply.c")
    if force or not os.path.exists(HOST_APPLY_LIB) or os.path.getmtime(ha) > os.path.getmtime(HOST_APPLY_LIB):
        subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", HOST_APPLY_LIB, ha], check=True)
    return LIB


def host_apply(ban_batch, log_path=None):
    """workloads/host_apply.c over a bjx_ban_batch (ctypes struct): the
    compiled stand-in for the Go host's Update per record + ban-log write.
    Returns (seconds, entries changed)."""
    L = C.CDLL(HOST_APPLY_LIB)
    L.bjx_host_apply.restype = C.c_double
    L.bjx_host_apply.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_uint64)]
    ch = C.c_uint64(0)
    secs = L.bjx_host_apply(C.addressof(ban_batch), log_path.encode() if log_path else None, C.byref(ch))
    return secs, ch.value


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.bjx_synth_host.restype = C.c_uint64
        L.bjx_synth_host.argtypes = [C.POINTER(SynthCfg), C.c_char_p, C.c_uint64]
        L.bjx_synth_device.restype = C.c_uint64
        L.bjx_synth_device.argtypes = [C.POINTER(SynthCfg), C.c_void_p, C.c_uint64, C.c_void_p]
        _lib = L
    return _lib


@dataclass(frozen=True)
class Workload:
    name: str
    description: str
    rules_yaml: str
    seed: int
    n_lines: int
    n_ips: int
    n_hosts: int
    other_host_pct: int = 20
    trigger_permille: int = 10
    ua_heavy: int = 0
    ipv6_pct: int = 2
    us_per_line: int = 10
    fixture_hosts: int = 0
    ip_mode: int = 0      # IP_UNIFORM / IP_ZIPF / IP_DISTINCT (workloads/synth.hip)
    zipf_milli: int = 1100
    hot_pct: int = 0      # share of lines from one DDoS IP (pool index 0)

    def synth_cfg(self, first_line=0, n_lines=None) -> SynthCfg:
        return SynthCfg(self.seed, first_line, self.n_lines if n_lines is None else n_lines, T0_MS,
                        self.us_per_line, self.n_ips, self.n_hosts, self.other_host_pct, self.trigger_permille,
                        self.ua_heavy, self.ipv6_pct, 3, self.fixture_hosts, self.ip_mode, self.zipf_milli,
                        self.hot_pct, 0)

    def host_lines(self, first_line=0, n_lines=None) -> bytes:
        cfg = self.synth_cfg(first_line, n_lines)
        need = lib().bjx_synth_host(C.byref(cfg), None, 0)
        buf = C.create_string_buffer(int(need) + 1)
        got = lib().bjx_synth_host(C.byref(cfg), buf, need + 1)
        return buf.raw[:got]

    def device_lines(self, device=0, first_line=0, n_lines=None):
        """Render straight into a torch uint8 tensor in HBM; returns (tensor, nbytes)."""
        import torch
        cfg = self.synth_cfg(first_line, n_lines)
        stream = torch.cuda.current_stream(device).cuda_stream
        need = lib().bjx_synth_device(C.byref(cfg), None, 0, C.c_void_p(stream))
        t = torch.empty(int(need) + 64, dtype=torch.uint8, device="cuda:%d" % device)
        got = lib().bjx_synth_device(C.byref(cfg), C.c_void_p(t.data_ptr()), need + 64, C.c_void_p(stream))
        if got != need:
            raise RuntimeError("synthetic generation failed")
        return t, int(need)

    def now_ns(self, first_line=0, n_lines=None) -> int:
        """Injected clock (time.Now() of consumeLine): the batch's first timestamp,
        so no line is more than 10 s old and OldLine never fires; later lines are
        in the future, as in the reference's own tests."""
        return (T0_MS * 1000 + first_line * self.us_per_line) // 1000 * 1_000_000


# --------------------------------------------------------------- rule sets

FIXTURE_RULES = """\
# fixtures/banjax-config-test.yaml (reference): the hot-path keys only
global_decision_lists:
  allow:
    - 20.20.20.20
  nginx_block:
    - 70.80.90.100
  challenge:
    - 8.8.8.8
    - 60.60.60.60
    - 192.168.1.0/24
per_site_decision_lists:
  example.com:
    allow:
      - 90.90.90.90
    challenge:
      - 91.91.91.91
  "localhost:8081":
    allow:
      - 90.90.90.90
      - 171.171.171.0/24
    challenge:
      - 91.91.91.91
      - 192.168.0.0/24
    nginx_block:
      - 92.92.92.92
per_site_regexes_with_rates:
  "localhost:8081":
    - decision: nginx_block
      hits_per_interval: 0
      interval: 1
      regex: .*block_local
      rule: "instant block_local"
regexes_with_rates:
  - decision: allow
    hits_per_interval: 0
    interval: 1
    regex: .*allowme.*
    rule: "unblock backdoor"
  - decision: nginx_block
    hits_per_interval: 0
    interval: 1
    regex: .*blockme.*
    rule: "instant block"
  - decision: challenge
    hits_per_interval: 0
    interval: 1
    regex: .*challengeme.*
    rule: "instant challenge"
expiring_decision_ttl_seconds: 10
"""

# banjax-config.yaml:59-95 style globals
_GLOBALS = """\
  - decision: nginx_block
    hits_per_interval: 800
    interval: 30
    regex: .*
    rule: "All sites/methods: 800 req/30 sec"
    hosts_to_skip:
      cdn0.other.net: true
      cdn1.other.net: true
      site007.example.com: true
  - decision: nginx_block
    hits_per_interval: 45
    interval: 60
    regex: "^POST .*"
    rule: "All sites/POST: 45 req/60 sec"
  - decision: allow
    hits_per_interval: 0
    interval: 1
    regex: .*allowme.*
    rule: "unblock backdoor"
  - decision: challenge
    hits_per_interval: 0
    interval: 1
    regex: .*challengeme.*
    rule: "instant challenge"
  - decision: iptables_block
    hits_per_interval: 0
    interval: 1
    regex: ".*banme.*"
    rule: "instant ban"
  - decision: nginx_block
    hits_per_interval: 0
    interval: 1
    regex: .*blockme.*
    rule: "instant block"
"""


def _q(s):
    return "'" + s.replace("'", "''") + "'"


def per_site_rules(n_hosts=100):
    """cfg3: 10 per-site rules for each of n_hosts hosts (1k rules at 100 hosts)."""
    out = ["per_site_regexes_with_rates:"]
    for h in range(n_hosts):
        host = "site%03d.example.com" % h
        hr = host.replace(".", r"\.")
        rules = [
            ("wp-login", r"GET %s GET \/wp-login\.php HTTP\/[0-2.]+ .*" % hr, 60, 20, "challenge"),
            ("xmlrpc", r"POST %s POST \/xmlrpc\.php" % hr, 60, 5, "nginx_block"),
            ("api burst", r"^GET %s GET \/api\/v1\/items\/[0-9]+ " % hr, 10, 50, "challenge"),
            ("admin", r"(GET|POST) \S+ (GET|POST) \/admin\/", 30, 10, "nginx_block"),
            ("sqli", r"(?i)union.+select", 1, 0, "iptables_block"),
            ("traversal", r"\.(php|asp|aspx|jsp)\?.*=(\.\.\/)+", 1, 0, "nginx_block"),
            ("env", r"\/\.env", 1, 0, "nginx_block"),
            ("search flood", r"GET \S+ GET \/search\?q=\w+ ", 5, 30, "challenge"),
            ("static", r"\/static\/(js|css)\/", 10, 400, "challenge"),
            ("bots", r"(?i)(ahrefs|semrush|mj12)bot", 60, 100, "challenge"),
        ]
        out.append("  %s:" % host)
        for name, rx, iv, hits, dec in rules:
            out.append("    - rule: %s\n      regex: %s\n      interval: %d\n      hits_per_interval: %d\n"
                       "      decision: %s" % (_q("%s %s" % (host, name)), _q(rx), iv, hits, dec))
    return "\n".join(out) + "\n"


def stress_global_rules(n_rules=100):
    """cfg2: TestPerSiteRegexStress-shaped global rules
    (regex_rate_limiter_test.go:317) over the generated hosts/paths."""
    paths = [r"\/wp-login\.php", r"\/xmlrpc\.php", r"\/about", r"\/contact", r"\/robots\.txt", r"\/index\.html"]
    out = ["regexes_with_rates:"]
    out.append(_GLOBALS.rstrip("\n"))
    k = 0
    while k < n_rules - 6:
        h = k // len(paths)
        p = paths[k % len(paths)]
        out.append("  - rule: 'rule%d'\n    regex: %s\n    interval: 1\n    hits_per_interval: 3\n"
                   "    decision: nginx_block" % (k, _q(r"GET site%03d\.example\.com GET %s HTTP\/[0-2.]+ .*" % (h, p))))
        k += 1
    return "\n".join(out) + "\n"


UA_RULES = """\
regexes_with_rates:
  - rule: "mac firefox"
    regex: 'Macintosh.*Firefox/\\d+'
    interval: 60
    hits_per_interval: 50
    decision: challenge
  - rule: "scrapers"
    regex: '(?i)scrapy|mechanize'
    interval: 10
    hits_per_interval: 5
    decision: nginx_block
  - rule: "ahrefs"
    regex: 'AhrefsBot'
    interval: 60
    hits_per_interval: 20
    decision: nginx_block
  - rule: "semrush"
    regex: 'SemrushBot'
    interval: 60
    hits_per_interval: 20
    decision: nginx_block
  - rule: "any firefox"
    regex: '.*Firefox/\\d+'
    interval: 30
    hits_per_interval: 200
    decision: challenge
"""

DDOS_RULES = """\
regexes_with_rates:
  - rule: "instant"
    regex: 'GET \\S+ GET \\/wp-login\\.php'
    interval: 1
    hits_per_interval: 0
    decision: nginx_block
  - rule: "burst2"
    regex: '^(GET|POST) \\S+ (GET|POST) \\/(api|search)'
    interval: 5
    hits_per_interval: 2
    decision: challenge
  - rule: "flood10"
    regex: '.*'
    interval: 60
    hits_per_interval: 10
    decision: iptables_block
"""

CFG1 = Workload("cfg1", "fixtures/banjax-config-test.yaml rules over 1M synthetic nginx lines, IPs Zipf(1.1) over 100k",
                FIXTURE_RULES, seed=1, n_lines=1_000_000, n_ips=100_000, n_hosts=32, trigger_permille=10,
                fixture_hosts=1, ip_mode=1)
REGEX_BANNER_RULES = """\
# fixtures/banjax-config-test-regex-banner.yaml (reference): the hot-path keys only
global_decision_lists:
  allow:
    - 20.20.20.20
    - 12.12.12.12
  iptables_block:
    - 30.40.50.60
  nginx_block:
    - 70.80.90.100
  challenge:
    - 8.8.8.8
per_site_decision_lists:
  example.com:
    allow:
      - 90.90.90.90
    challenge:
      - 91.91.91.91
  "localhost:8081":
    allow:
      - 90.90.90.90
    challenge:
      - 91.91.91.91
    nginx_block:
      - 92.92.92.92
per_site_regexes_with_rates: {}
regexes_with_rates:
  - decision: allow
    hits_per_interval: 0
    interval: 1
    regex: .*allowme.*
    rule: "unblock backdoor"
  - decision: nginx_block
    hits_per_interval: 0
    interval: 1
    regex: .*blockme.*
    rule: "instant block"
  - decision: challenge
    hits_per_interval: 0
    interval: 1
    regex: .*challengeme.*
    rule: "instant challenge"
  - decision: challenge
    hits_per_interval: 0
    interval: 1
    regex: .*
    rule: "Challenge all but skip localhost:8081"
    hosts_to_skip:
      "localhost:8081": true
  - decision: nginx_block
    hits_per_interval: 45
    interval: 60
    regex: "GET .* /"
    rule: "All sites/GET: 45 req/60 sec"
expiring_decision_ttl_seconds: 10
"""

RELOAD_RULES = """\
# fixtures/banjax-config-test-reload.yaml (reference): the hot-path keys only
global_decision_lists:
  allow: []
  iptables_block:
    - 30.40.50.60
  nginx_block:
    - 70.80.90.100
  challenge:
    - 20.20.20.20
per_site_decision_lists:
  example.com:
    allow:
      - 90.90.90.90
    challenge:
      - 91.91.91.91
  "localhost:8081":
    allow:
      - 91.91.91.91
    challenge: []
    nginx_block:
      - 92.92.92.92
per_site_regexes_with_rates: {}
regexes_with_rates:
  - decision: allow
    hits_per_interval: 0
    interval: 1
    regex: .*allowme.*
    rule: "unblock backdoor"
  - decision: nginx_block
    hits_per_interval: 0
    interval: 1
    regex: .*blockme.*
    rule: "instant block"
expiring_decision_ttl_seconds: 10
"""


def standalone_line(t_s: int, ip: str, path: str, host: str = "localhost:8081", method: str = "GET",
                    ua: str = "Go-http-client/1.1") -> bytes:
    """The log line banjax's standalone-testing middleware writes for each
    integration-test request (reference internal/http_server.go:150-167):
    '%f %s %s %s %s %s HTTP/1.1 %s' of float64(Unix seconds), X-Client-IP,
    method, Host, method, the `path` query value, User-Agent."""
    return ("%f %s %s %s %s %s HTTP/1.1 %s\n" % (float(t_s), ip, method, host, method, path, ua)).encode()


CFG2 = Workload("cfg2", "100 global rules (TestPerSiteRegexStress shape + banjax-config.yaml globals), 100M lines, 1M IPs",
                stress_global_rules(100) + "expiring_decision_ttl_seconds: 10\n",
                seed=2, n_lines=100_000_000, n_ips=1_000_000, n_hosts=100)
CFG3 = Workload("cfg3", "1k per-site rules (100 hosts x 10, host-filtered) + 6 globals; 125M lines per GPU (1B at 8 GPUs)",
                "regexes_with_rates:\n" + _GLOBALS + per_site_rules(100) + "expiring_decision_ttl_seconds: 10\n",
                seed=3, n_lines=125_000_000, n_ips=1_000_000, n_hosts=100)
CFG4 = Workload("cfg4", "UA-heavy 2-8 KB lines, user-agent regexes (fixtures/banjax-config-test-ua.yaml style)",
                UA_RULES + "expiring_decision_ttl_seconds: 10\n",
                seed=4, n_lines=2_000_000, n_ips=100_000, n_hosts=32, ua_heavy=1)
CFG5 = Workload("cfg5", "DDoS burst: 100M distinct IPs (one line each), high trip rate",
                DDOS_RULES + "expiring_decision_ttl_seconds: 10\n",
                seed=5, n_lines=100_000_000, n_ips=100_000_000, n_hosts=32, trigger_permille=50, ip_mode=2)
CFG5H = Workload("cfg5h", "DDoS hot key: one IP sends 25% of 100M lines, the rest Zipf(1.1) over 10M IPs",
                 DDOS_RULES + "expiring_decision_ttl_seconds: 10\n",
                 seed=6, n_lines=100_000_000, n_ips=10_000_000, n_hosts=32, trigger_permille=50, ip_mode=1, hot_pct=25)

# not a BASELINE config: the reference's TestPerSiteRegexStress shape at 1,000
# global rules, so every line's scope has 1,000 positions (past the 128 of
# k_lines2's decision tables: the per-line pass is k_lines)
CFG2K = Workload("cfg2k", "1k global rules (TestPerSiteRegexStress shape: every line's scope 1,000 rules), 20M lines, 1M IPs",
                 stress_global_rules(1000) + "expiring_decision_ttl_seconds: 10\n",
                 seed=7, n_lines=20_000_000, n_ips=1_000_000, n_hosts=100)

ALL = {w.name: w for w in (CFG1, CFG2, CFG3, CFG4, CFG5, CFG5H, CFG2K)}


def scaled(w: Workload, n_lines: int, n_ips=None) -> Workload:
    return replace(w, n_lines=n_lines, n_ips=n_ips if n_ips is not None else min(w.n_ips, max(1, n_lines // 4)))
