"""Generate the Unicode data headers shared by the rule compiler and the oracle.

  third_party/unicode/fold_orbits.h     unicode.SimpleFold orbits ((?i) folding)
  third_party/unicode/unicode_tables.h  general categories and scripts (\\p{..})

Go 1.25 (the reference's toolchain, go.mod:3) ships Unicode 15.0.0 tables in
package unicode; regexp/syntax reads them for (?i) (SimpleFold) and for the
UnicodeGroups flag of syntax.Perl (\\pL, \\p{Greek}, ...; regexp.Compile at
reference internal/config.go:110).  No Go tables exist offline, so the data is
rebuilt here from two independent sources present in the image:

  * ICU 70 (libicuuc.so.70, Unicode 14.0): every code point assigned in <= 14.0
    (u_charAge), its general category (u_charType), script (uscript_getScript)
    and simple case mappings (u_tolower / u_toupper / u_totitle / u_foldCase);
  * the Unicode 15.0 additions (DerivedAge.txt "15.0" lines, DELTA_15 below,
    4,488 code points), whose category and script come from the `regex`
    module's Unicode database; the script checks that ICU has none of them and
    that `regex` has all of them.

Unicode 15.0 added no case pairs; the script checks that too, by rebuilding the
orbits from the `regex` module's (?i) matching over every cased code point of
<= 15.0 and requiring the same orbits.  Data only: no code of the reference or
of Go is involved.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT_DIR = os.path.join(ROOT, "third_party", "unicode")
MAX = 0x110000

# DerivedAge.txt, Age=15.0 (Unicode 15.0.0, September 2022)
DELTA_15 = [
    (0x0CF3, 0x0CF3), (0x0ECE, 0x0ECE), (0x10EFD, 0x10EFF), (0x1123F, 0x11241), (0x11B00, 0x11B09),
    (0x11F00, 0x11F10), (0x11F12, 0x11F3A), (0x11F3E, 0x11F59), (0x1342F, 0x1342F), (0x13439, 0x1343F),
    (0x13440, 0x13455), (0x1B132, 0x1B132), (0x1B155, 0x1B155), (0x1D2C0, 0x1D2D3), (0x1DF25, 0x1DF2A),
    (0x1E030, 0x1E06D), (0x1E08F, 0x1E08F), (0x1E4D0, 0x1E4F9), (0x1F6DC, 0x1F6DC), (0x1F774, 0x1F776),
    (0x1F77B, 0x1F77F), (0x1F7D9, 0x1F7D9), (0x1FA75, 0x1FA77), (0x1FA87, 0x1FA88), (0x1FAAD, 0x1FAAF),
    (0x1FABB, 0x1FABD), (0x1FABF, 0x1FABF), (0x1FACE, 0x1FACF), (0x1FADA, 0x1FADB), (0x1FAE8, 0x1FAE8),
    (0x1FAF7, 0x1FAF8), (0x31350, 0x323AF),
]

# ICU UCharCategory -> Unicode general category
ICU_GC = ["Cn", "Lu", "Ll", "Lt", "Lm", "Lo", "Mn", "Me", "Mc", "Nd", "Nl", "No", "Zs", "Zl", "Zp", "Cc", "Cf",
          "Co", "Cs", "Pd", "Ps", "Pe", "Pc", "Po", "Sm", "Sc", "Sk", "So", "Pi", "Pf"]
BASE_GC = [g for g in ICU_GC]
# Go package unicode's composite categories (C is Cc|Cf|Co|Cs: unassigned code
# points are in no table of Go's, only in Cn)
COMPOSITE = {
    "C": ["Cc", "Cf", "Co", "Cs"], "L": ["Lu", "Ll", "Lt", "Lm", "Lo"], "LC": ["Lu", "Ll", "Lt"],
    "M": ["Mn", "Mc", "Me"], "N": ["Nd", "Nl", "No"], "P": ["Pc", "Pd", "Ps", "Pe", "Pi", "Pf", "Po"],
    "S": ["Sm", "Sc", "Sk", "So"], "Z": ["Zs", "Zl", "Zp"],
}
# PropertyValueAliases.txt, gc (unicode.CategoryAliases)
CAT_ALIASES = {
    "Cased_Letter": "LC", "Close_Punctuation": "Pe", "Combining_Mark": "M", "Connector_Punctuation": "Pc",
    "Control": "Cc", "Currency_Symbol": "Sc", "Dash_Punctuation": "Pd", "Decimal_Number": "Nd",
    "Enclosing_Mark": "Me", "Final_Punctuation": "Pf", "Format": "Cf", "Initial_Punctuation": "Pi",
    "Letter": "L", "Letter_Number": "Nl", "Line_Separator": "Zl", "Lowercase_Letter": "Ll", "Mark": "M",
    "Math_Symbol": "Sm", "Modifier_Letter": "Lm", "Modifier_Symbol": "Sk", "Nonspacing_Mark": "Mn",
    "Number": "N", "Open_Punctuation": "Ps", "Other": "C", "Other_Letter": "Lo", "Other_Number": "No",
    "Other_Punctuation": "Po", "Other_Symbol": "So", "Paragraph_Separator": "Zp", "Private_Use": "Co",
    "Punctuation": "P", "Separator": "Z", "Space_Separator": "Zs", "Spacing_Mark": "Mc", "Surrogate": "Cs",
    "Symbol": "S", "Titlecase_Letter": "Lt", "Unassigned": "Cn", "Uppercase_Letter": "Lu", "cntrl": "Cc",
    "digit": "Nd", "punct": "P",
}
POST_15_ORBITS = {(0x390, 0x1FD3), (0x3B0, 0x1FE3), (0xFB05, 0xFB06)}
# U+0130 / U+0131 fold only under Turkic rules, which simple folding excludes
TURKIC_ONLY = {0x130, 0x131}


def icu():
    L = C.CDLL("libicuuc.so.70")
    for fn, res, args in [("u_charType_70", C.c_int8, [C.c_int32]), ("uscript_getScript_70", C.c_int, [C.c_int32, C.POINTER(C.c_int)]),
                          ("uscript_getName_70", C.c_char_p, [C.c_int]), ("u_tolower_70", C.c_int32, [C.c_int32]),
                          ("u_toupper_70", C.c_int32, [C.c_int32]), ("u_totitle_70", C.c_int32, [C.c_int32]),
                          ("u_foldCase_70", C.c_int32, [C.c_int32, C.c_uint32]),
                          ("u_charAge_70", None, [C.c_int32, C.c_uint8 * 4]),
                          ("u_getUnicodeVersion_70", None, [C.c_uint8 * 4])]:
        f = getattr(L, fn)
        f.restype = res
        f.argtypes = args
    v = (C.c_uint8 * 4)()
    L.u_getUnicodeVersion_70(v)
    assert tuple(v[:2]) == (14, 0), tuple(v)
    return L


def ranges_of(cps):
    out = []
    for c in sorted(cps):
        if out and out[-1][1] + 1 == c:
            out[-1][1] = c
        else:
            out.append([c, c])
    return [tuple(r) for r in out]


def main():
    import regex
    L = icu()
    err = C.c_int(0)
    gc = [None] * MAX
    sc = [None] * MAX
    age = (C.c_uint8 * 4)()
    for cp in range(MAX):
        t = ICU_GC[L.u_charType_70(cp)]
        gc[cp] = t
        if t != "Cn":
            s = L.uscript_getScript_70(cp, C.byref(err))
            sc[cp] = L.uscript_getName_70(s).decode()
    # Unicode 15.0 additions: absent from ICU 70, present in `regex`
    gc_names = sorted(set(ICU_GC) - {"Cn"})
    pats = {g: regex.compile(r"\p{gc=%s}" % g) for g in gc_names}
    scripts_regex = sorted(set(s for s in sc if s))
    added_scripts = ["Kawi", "Nag_Mundari"]
    spats = {s: regex.compile(r"\p{sc=%s}" % s) for s in scripts_regex + added_scripts}
    n15 = 0
    for lo, hi in DELTA_15:
        for cp in range(lo, hi + 1):
            L.u_charAge_70(cp, age)
            assert gc[cp] == "Cn" and tuple(age) == (0, 0, 0, 0), "U+%04X assigned in ICU 70" % cp
            ch = chr(cp)
            g = [k for k, p in pats.items() if p.match(ch)]
            assert len(g) == 1, ("U+%04X" % cp, g)
            s = [k for k, p in spats.items() if p.match(ch)]
            assert len(s) == 1, ("U+%04X" % cp, s)
            gc[cp], sc[cp] = g[0], s[0]
            n15 += 1
    assert n15 == 4488, n15
    # ---- simple fold orbits (ICU 70 mappings)
    parent = {}

    def find(x):
        while parent.get(x, x) != x:
            x = parent[x]
        return x

    def union(a, b):
        parent.setdefault(a, a)
        parent.setdefault(b, b)
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)

    for cp in range(MAX):
        if 0xD800 <= cp <= 0xDFFF or cp in TURKIC_ONLY or gc[cp] == "Cn":
            continue
        for m in (L.u_tolower_70(cp), L.u_toupper_70(cp), L.u_totitle_70(cp), L.u_foldCase_70(cp, 0)):
            if m != cp and m not in TURKIC_ONLY:
                union(cp, m)
    orbits = {}
    for cp in parent:
        orbits.setdefault(find(cp), []).append(cp)
    orbit_sets = sorted(tuple(sorted(m)) for m in orbits.values() if len(m) > 1)
    # cross-check: the `regex` module's (?i) equivalence over the same code points
    cased = [cp for cp in range(MAX) if gc[cp] != "Cn" and not (0xD800 <= cp <= 0xDFFF)
             and (cp in parent or regex.match(r"\p{Cased}|\p{CWCF}|\p{CWCM}", chr(cp)))]
    hay = "".join(chr(c) for c in cased)
    seen, rx_orbits = set(), []
    for cp in cased:
        if cp in seen or cp in TURKIC_ONLY:
            continue
        mem = sorted(set(ord(x) for x in regex.findall(r"(?i)" + regex.escape(chr(cp)), hay)) - TURKIC_ONLY)
        seen.update(mem)
        if len(mem) > 1:
            rx_orbits.append(tuple(mem))
    # CaseFolding.txt gained simple foldings for U+1FD3, U+1FE3 and U+FB05 after
    # 15.0 (the `regex` module carries a newer database): not in Go 1.25
    rx_orbits = sorted(o for o in rx_orbits if o not in POST_15_ORBITS)
    if rx_orbits != orbit_sets:
        a, b = set(orbit_sets), set(rx_orbits)
        raise SystemExit("fold orbits differ: icu-only %s regex-only %s" % (sorted(a - b)[:8], sorted(b - a)[:8]))
    pairs = []
    for m in orbit_sets:
        for i, x in enumerate(m):
            pairs.append((x, m[(i + 1) % len(m)]))
    pairs.sort()
    with open(os.path.join(OUT_DIR, "fold_orbits.h"), "w") as f:
        f.write("/* Generated by tools/gen_unicode_tables.py: Unicode 15.0.0 simple case-fold orbits\n"
                " * (ICU 70 / Unicode 14.0 case mappings; Unicode 15.0 added no case pairs, checked\n"
                " * against the `regex` module's (?i) equivalence).  SimpleFold(r): next member of\n"
                " * r's orbit (wrapping); runes not listed fold to themselves.  Data only. */\n")
        f.write("#pragma once\n#include <stdint.h>\n#define BJX_UNICODE_VERSION \"15.0.0\"\n")
        f.write("#define BJX_FOLD_N %d\n" % len(pairs))
        for nm, k in (("bjx_fold_from", 0), ("bjx_fold_to", 1)):
            f.write("static const uint32_t %s[BJX_FOLD_N] = {\n" % nm)
            for i in range(0, len(pairs), 12):
                f.write("  " + ",".join("0x%x" % p[k] for p in pairs[i:i + 12]) + ",\n")
            f.write("};\n")
    # ---- category and script tables
    tables = []  # (kind, name, ranges)
    by_gc = {}
    for cp in range(MAX):
        by_gc.setdefault(gc[cp], []).append(cp)
    for g in BASE_GC:
        tables.append(("cat", g, ranges_of(by_gc.get(g, []))))
    for g, parts in COMPOSITE.items():
        cps = []
        for p in parts:
            cps.extend(by_gc.get(p, []))
        tables.append(("cat", g, ranges_of(cps)))
    by_sc = {}
    for cp in range(MAX):
        if sc[cp] and sc[cp] != "Unknown":
            by_sc.setdefault(sc[cp], []).append(cp)
    for s in sorted(by_sc):
        tables.append(("script", s, ranges_of(by_sc[s])))
    flat, index = [], []
    for kind, name, rs in tables:
        index.append((kind, name, len(flat) // 2, len(rs)))
        for lo, hi in rs:
            flat += [lo, hi]
    with open(os.path.join(OUT_DIR, "unicode_tables.h"), "w") as f:
        f.write("/* Generated by tools/gen_unicode_tables.py: Unicode 15.0.0 general categories and\n"
                " * scripts as Go's package unicode defines them (Categories incl. LC and Cn, Scripts,\n"
                " * CategoryAliases), for regexp/syntax UnicodeGroups (\\p{..}).  Sources: ICU 70\n"
                " * (Unicode 14.0) + the Unicode 15.0 DerivedAge additions.  Data only. */\n")
        f.write("#pragma once\n#include <stdint.h>\n")
        f.write("typedef struct { const char *name; uint32_t kind, off, n; } bjx_uni_table; /* kind 0 category, 1 script */\n")
        f.write("#define BJX_UNI_NTABLES %d\n#define BJX_UNI_NRANGES %d\n" % (len(index), len(flat) // 2))
        f.write("static const uint32_t bjx_uni_ranges[2 * BJX_UNI_NRANGES] = {\n")
        for i in range(0, len(flat), 12):
            f.write("  " + ",".join("0x%x" % x for x in flat[i:i + 12]) + ",\n")
        f.write("};\nstatic const bjx_uni_table bjx_uni_tables[BJX_UNI_NTABLES] = {\n")
        for kind, name, off, n in index:
            f.write("  {\"%s\", %d, %d, %d},\n" % (name, 0 if kind == "cat" else 1, off, n))
        f.write("};\n#define BJX_UNI_NALIASES %d\n" % len(CAT_ALIASES))
        f.write("static const char *const bjx_uni_cat_aliases[2 * BJX_UNI_NALIASES] = {\n")
        for a, t in sorted(CAT_ALIASES.items()):
            f.write("  \"%s\", \"%s\",\n" % (a, t))
        f.write("};\n")
    print("fold pairs %d, tables %d, ranges %d, 15.0 additions %d" % (len(pairs), len(index), len(flat) // 2, n15))


if __name__ == "__main__":
    main()
