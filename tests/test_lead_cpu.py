"""Bounded lead distance of prefilter rules (regex_compiler.cpp
bounded_leading_literals): every match begins at most `dist` bytes before an
occurrence of the rule's literals, so a DFA job may start `dist + 3` bytes
before the first hit instead of at rest[0] (engine.hip lead_start).  Checked
here on the host: the rule's compiled DFA started there decides every text as
the oracle (Go regexp restated) does on the whole text."""
import random

import pytest

from banjax_amd import _lib
from tests.test_cpu_boundary import _one_rule_ruleset
from oracle import oracle as O

# pattern, expected lead distance (-1: not a bounded-lead rule), its literals (text, case-insensitive)
CASES = [
    (r"(?i)scrapy|mechanize", 4, [("crapy", True), ("mechanize", True)]),
    (r"x[0-9]{2}abcd", 3, [("abcd", False)]),
    (r"[a-z]{1,4}=token", 4, [("=token", False)]),
    (r"é{2}wxyz", 4, [("wxyz", False)]),
    (r"(?:ab|cde)wxyz1", 0, [("abwxyz1", False), ("cdewxyz1", False)]),
    (r"Macintosh.*Firefox/\d+", 0, [("Macintosh", False)]),
    (r"\d+abcd", -1, []),
    (r"\babcd", -1, []),
    (r"(?:x|^y)abcd", -1, []),
]


def _first_hit(text, lits):
    best = None
    low = text.lower()
    for s, ci in lits:
        hay, needle = (low, s.lower().encode()) if ci else (text, s.encode())
        i = hay.find(needle)
        if i >= 0 and (best is None or i < best):
            best = i
    return best


@pytest.mark.parametrize("pat,dist,lits", CASES)
def test_lead_distance_and_soundness(pat, dist, lits):
    rs = _one_rule_ruleset(pat)
    L = _lib.lib()
    assert L.bjx_debug_rule_lead(rs.handle, 0) == dist, pat
    if dist < 0:
        return
    ore = O.Regex(pat)
    rnd = random.Random(hash(pat) & 0xFFFF)
    frags = [b"a", b"b", b"x", b"1", b"22", b" ", b"=", b"\xc3\xa9", b"\xc5\xbf", b"\xe2\x84\xaa", b"\xff", b"\xc3",
             b"S", b"s", b"z"] + [s.encode() for s, _ in lits] + [s.upper().encode() for s, _ in lits]
    for _ in range(1500):
        t = b"".join(rnd.choice(frags) for _ in range(rnd.randrange(0, 14)))
        f = _first_hit(t, lits)
        want = ore.match(t)
        if f is None:
            assert not want, (pat, t)  # no literal, no match: the job starts at the end
            continue
        p = max(0, f - dist - 3)
        got = L.bjx_debug_rule_match_host(rs.handle, 0, t[p:], len(t) - p)
        assert got == int(want), (pat, t, p)
