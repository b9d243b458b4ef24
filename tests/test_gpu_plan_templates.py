"""GPU parity for the LDS plan classes (decide_plan_lds): per-site rules whose
literal spells the site's own host (A + host + C templates, shared by every
host), the host spelled away from the host field, near-miss hosts, case-
insensitive host parts (no template: per-host class), hosts spelled twice, and
anchored templates — engine vs the oracle, bit-exact.  Reference semantics:
internal/regex_rate_limiter.go:175-211 (per-site rules of the line's host)."""
import random

import pytest

from tests.parity import Pair

pytestmark = pytest.mark.gpu
S = 1_000_000_000

HOSTS = ["a.example.com", "bb.example.org", "c-3.net", "Mixed.Case.Host", "d.io"]


def _rules():
    out = ["regexes_with_rates:",
           "  - rule: 'all'\n    regex: '.*'\n    interval: 60\n    hits_per_interval: 100000\n    decision: challenge",
           "per_site_regexes_with_rates:"]
    for i, h in enumerate(HOSTS):
        e = h.replace(".", r"\.")
        rules = [
            ("wp", r"GET %s GET \/wp-login\.php" % e, 60, 3),                  # template, piece = C, equivalent
            ("wp2", r"GET %s GET \/wp-login\.php HTTP\/[0-2.]+ .*" % e, 60, 2),  # template, DFA after the check
            ("api", r"^GET %s GET \/api\/[0-9]+ " % e, 10, 2),                  # anchored template
            ("xml", r"^POST %s POST \/xmlrpc\.php" % e, 10, 1),                  # anchored template, equivalent
            ("pre", r"zz-%s-yy" % e, 10, 1),                                    # A and C both short
            ("head", r"%s\/login-form-page" % e, 10, 1),                        # piece = C, empty A
            ("tail", r"xx-long-prefix-piece %s" % e, 10, 1),                     # piece = A, empty C
            ("ci", r"(?i)get %s get \/ci" % e, 10, 1),                          # case-insensitive host: no template
            ("twice", r"%s GET \/%s" % (e, e), 10, 1),                          # host twice: no template
            ("admin", r"(GET|POST) \S+ (GET|POST) \/admin\/", 30, 2),            # shared pattern
        ]
        if i == 2:
            rules = rules[::-1]   # another order: another class
        out.append("  %s:" % h)
        for name, rx, iv, hits in rules:
            out.append("    - rule: '%s %s'\n      regex: '%s'\n      interval: %d\n      hits_per_interval: %d\n"
                       "      decision: nginx_block" % (h, name, rx.replace("'", "''"), iv, hits))
    return "\n".join(out) + "\nexpiring_decision_ttl_seconds: 10\n"


def _lines(rnd, t, n):
    hosts = HOSTS + ["a.example.co", "a.example.comm", "xa.example.com", "mixed.case.host", "other.net"]
    frags = []
    for h in HOSTS + ["a.example.co", "mixed.case.host"]:
        frags += ["GET %s GET /wp-login.php" % h, "GET %s GET /wp-login.php HTTP/1.1 ua" % h, "zz-%s-yy" % h,
                  "%s/login-form-page" % h, "xx-long-prefix-piece %s" % h, "get %s get /ci" % h.upper(),
                  "%s GET /%s" % (h, h), "GET %s GET /api/12 " % h]
    frags += ["/admin/", "GET /x", "-", "ua/1.0", "xmlrpc.php"]
    out = []
    for j in range(n):
        h = rnd.choice(hosts)
        m = rnd.choice(["GET", "POST", "GET", "PUT"])
        path = rnd.choice(["/wp-login.php HTTP/1.1", "/api/%d HTTP/1.1" % rnd.randrange(100), "/xmlrpc.php",
                           "/admin/x", "/login-form-page", "/q?u=" + rnd.choice(frags).replace(" ", "%20"), "/"])
        tail = " ".join(rnd.choice(frags) for _ in range(rnd.randrange(0, 3)))
        out.append(("%d 10.0.%d.%d %s %s %s %s %s" % (t, j % 7, j % 13, m, h, m, path, tail)).encode())
    return b"\n".join(out) + b"\n"


@pytest.mark.parametrize("seed", [1, 2])
def test_plan_templates(seed):
    rnd = random.Random(seed)
    t = 1700000000
    pair = Pair(_rules())
    pair.feed(_lines(rnd, t, 6000), t * S)
    pair.feed(_lines(rnd, t + 1, 6000), (t + 1) * S)
    pair.compare_state(["10.0.1.1", "10.0.3.5"])
    pair.engine.close()
