"""The baked Unicode tables of the engine checked against an INDEPENDENT
source: Python's `unicodedata` (UCD 13.0.0), which shares nothing with
oracle/go_unicode.py (the `regex` module's 17.0 data cut back to 15.0) that
generated them.

Go 1.22 (go.mod:3-5) carries Unicode 15.0.0; its regexp \\p{..} classes are
unicode.Categories / unicode.Scripts, (?i) uses simple case folding orbits
(unicode.SimpleFold) and bytes.ToLower / strings.ToLower (the MatchKeywords
gate, pkg/fanal/secret/scanner.go:169-181) use unicode.ToLower.  For every
code point ASSIGNED in 13.0 these properties are checked here against
unicodedata; code points assigned later (14.0 / 15.0, and the post-15.0 ones
DESIGN.md "Unicode classes" lists) are outside what 13.0 can say.

* general categories: each assigned 13.0 code point is in exactly the table of
  its 13.0 category (and its one-letter major), except the few whose category
  Unicode changed between 13.0 and 15.0 (listed, with their 13.0 value);
* scripts: every letter whose 13.0 character NAME starts with a script's name
  is in that script's table (names are assigned with the script; no script
  data exists in unicodedata, so this is the independent evidence there is);
* ToLower: kLowerMap equals str.lower() wherever that is one character (the
  simple mapping; the only 13.0 code point with a longer full lowercase is
  U+0130, whose simple lowercase is U+0069);
* fold orbits: two code points share a kFoldOrbit orbit iff their str.casefold()
  agree, wherever that is one character (full folding = simple folding there).
"""
import os
import re
import unicodedata

import pytest

CSRC = os.path.join(os.path.dirname(__file__), "..", "trivy_amd", "csrc")
MAX = 0x110000

pytestmark = pytest.mark.skipif(unicodedata.unidata_version != "13.0.0",
                                reason="the independent source is Python 3.10's UCD 13.0.0")


def _read(name):
    return open(os.path.join(CSRC, name)).read()


def _uni_tables():
    txt = _read("gre_unicode_tables.h")
    idx = re.findall(r'\{"(\w+)", (\d+), (\d+)\}', txt)
    body = txt[txt.index("kUniRanges"):]
    rng = [(int(a, 16), int(b, 16)) for a, b in re.findall(r"\{0x([0-9a-fA-F]+), 0x([0-9a-fA-F]+)\}", body)]
    out = {}
    for name, off, n in idx:
        s = set()
        for lo, hi in rng[int(off):int(off) + int(n)]:
            s.update(range(lo, hi + 1))
        out[name] = s
    return out


def _pairs(name, table):
    txt = _read(name)
    body = txt[txt.index(table):]
    return [(int(a, 16), int(b, 16)) for a, b in re.findall(r"\{0x([0-9a-fA-F]+), 0x([0-9a-fA-F]+)\}", body)]


_T = None


def tables():
    global _T
    if _T is None:
        _T = _uni_tables()
    return _T


def assigned13():
    return [c for c in range(MAX) if unicodedata.category(chr(c)) != "Cn"]


# general-category changes between 13.0 and 15.0 (Unicode 14.0 UnicodeData
# changes: U+0295 is no longer a cased letter; two dependent vowel signs became
# spacing marks), as (13.0 value, the tables' value); any other difference
# fails the test.  Which release made them is not independently pinned here.
CAT_CHANGED = {0x0295: ("Ll", "Lo"), 0x1734: ("Mn", "Mc"), 0x1171E: ("Mn", "Mc")}


def test_categories_match_ucd13_for_every_assigned_code_point():
    T = tables()
    subcats = [n for n in T if len(n) == 2 and n[0] in "CLMNPSZ"]
    assert len(subcats) == 29
    owner = {}
    for name in subcats:
        for c in T[name]:
            assert c not in owner, f"U+{c:04X} in {owner.get(c)} and {name}"
            owner[c] = name
    bad = []
    for c in assigned13():
        cat = unicodedata.category(chr(c))
        got = owner.get(c)
        if got != cat and CAT_CHANGED.get(c) != (cat, got):
            bad.append((hex(c), cat, got))
        if got:
            assert c in T[got[0]], f"U+{c:04X}: {got} but not in major {got[0]}"
    assert not bad, f"{len(bad)} code points differ from UCD 13.0, first: {bad[:20]}"
    # majors are exactly the unions of their subcategories (Go's "C" has no Cn)
    for m in "CLMNPSZ":
        assert T[m] == set().union(*(T[s] for s in subcats if s[0] == m)), m


# script name -> the character-name prefix that the UCD gives its letters
SCRIPT_PREFIX = {
    "Latin": "LATIN ", "Greek": "GREEK ", "Cyrillic": "CYRILLIC ", "Armenian": "ARMENIAN ",
    "Hebrew": "HEBREW ", "Arabic": "ARABIC ", "Syriac": "SYRIAC ", "Thaana": "THAANA ",
    "Devanagari": "DEVANAGARI ", "Bengali": "BENGALI ", "Gurmukhi": "GURMUKHI ", "Gujarati": "GUJARATI ",
    "Oriya": "ORIYA ", "Tamil": "TAMIL ", "Telugu": "TELUGU ", "Kannada": "KANNADA ",
    "Malayalam": "MALAYALAM ", "Sinhala": "SINHALA ", "Thai": "THAI ", "Lao": "LAO ", "Tibetan": "TIBETAN ",
    "Myanmar": "MYANMAR ", "Georgian": "GEORGIAN ", "Hangul": "HANGUL ", "Ethiopic": "ETHIOPIC ",
    "Cherokee": "CHEROKEE ", "Ogham": "OGHAM ", "Runic": "RUNIC ", "Khmer": "KHMER ",
    "Mongolian": "MONGOLIAN ", "Hiragana": "HIRAGANA ", "Katakana": "KATAKANA ", "Bopomofo": "BOPOMOFO ",
    "Han": "CJK UNIFIED IDEOGRAPH-", "Yi": "YI SYLLABLE ", "Gothic": "GOTHIC ", "Deseret": "DESERET ",
    "Tagalog": "TAGALOG ", "Limbu": "LIMBU ", "Tai_Le": "TAI LE ", "Linear_B": "LINEAR B ",
    "Ugaritic": "UGARITIC ", "Shavian": "SHAVIAN ", "Osmanya": "OSMANYA ", "Cypriot": "CYPRIOT ",
    "Buginese": "BUGINESE ", "Coptic": "COPTIC ", "Glagolitic": "GLAGOLITIC ", "Tifinagh": "TIFINAGH ",
    "Balinese": "BALINESE ", "Cuneiform": "CUNEIFORM ", "Phoenician": "PHOENICIAN ", "Vai": "VAI ",
    "Javanese": "JAVANESE ", "Egyptian_Hieroglyphs": "EGYPTIAN HIEROGLYPH ", "Tangut": "TANGUT IDEOGRAPH-",
    "Adlam": "ADLAM ", "Osage": "OSAGE ", "Wancho": "WANCHO ", "Yezidi": "YEZIDI ",
}


# letters named after a script that Scripts.txt nevertheless puts in Common
# (shared punctuation-like modifier letters): checked as Common members
NAME_EXCEPTIONS = {0x0374: "Common",   # GREEK NUMERAL SIGN
                   0x0640: "Common",   # ARABIC TATWEEL
                   0xA9CF: "Common"}   # JAVANESE PANGRANGKEP


def test_script_letters_by_character_name():
    T = tables()
    checked = 0
    bad = []
    for c in assigned13():
        ch = chr(c)
        if not unicodedata.category(ch).startswith("L"):
            continue
        name = unicodedata.name(ch, "")
        for script, prefix in SCRIPT_PREFIX.items():
            if name.startswith(prefix):
                checked += 1
                want = NAME_EXCEPTIONS.get(c, script)
                if c not in T[want] or (want != script and c in T[script]):
                    bad.append((hex(c), name, want))
    assert checked > 100000
    assert not bad, f"{len(bad)} letters missing from their script, first: {bad[:20]}"


def test_to_lower_matches_ucd13_simple_lowercase():
    lower = dict(_pairs("gre_lower_table.h", "kLowerMap"))
    bad = []
    for c in assigned13():
        full = chr(c).lower()
        want = ord(full) if len(full) == 1 else (0x69 if c == 0x130 else None)
        if want is None:  # only U+0130 has a multi-character full lowercase in 13.0
            bad.append((hex(c), "multi-char lowercase"))
            continue
        if lower.get(c, c) != want:
            bad.append((hex(c), hex(lower.get(c, c)), hex(want)))
    assert not bad, f"{len(bad)} differ, first: {bad[:20]}"
    # the table maps only code points that change (and only assigned ones)
    for c, l in lower.items():
        assert c != l


def test_simple_fold_orbits_match_ucd13_case_folding():
    orbit_next = dict(_pairs("gre_fold_table.h", "kFoldOrbit"))
    # orbit id = the smallest member, by walking the ring
    orbit = {}
    for c in orbit_next:
        if c in orbit:
            continue
        ring, x = [c], orbit_next[c]
        while x != c:
            ring.append(x)
            x = orbit_next[x]
            assert len(ring) < 8
        for x in ring:
            orbit[x] = min(ring)
    by_fold = {}
    for c in assigned13():
        f = chr(c).casefold()
        if len(f) == 1:
            by_fold.setdefault(f, set()).add(c)
    bad = []
    for f, members in by_fold.items():
        ids = {orbit.get(c, c) for c in members}
        if len(ids) != 1:
            bad.append((f, sorted(hex(c) for c in members), ids))
    assert not bad, f"{len(bad)} casefold classes split across orbits, first: {bad[:10]}"
    # and no orbit joins two different single-character foldings
    folds_of = {}
    for c, oid in orbit.items():
        if unicodedata.category(chr(c)) == "Cn":
            continue
        f = chr(c).casefold()
        if len(f) == 1:
            folds_of.setdefault(oid, set()).add(f)
    assert all(len(v) == 1 for v in folds_of.values())


def test_post_13_code_points_in_the_tables_are_bounded():
    """Code points the tables hold that UCD 13.0 leaves unassigned: Unicode
    14.0 and 15.0 additions (in Go 1.22) plus the post-15.0 additions to
    older scripts that the oracle cannot cut (DESIGN.md lists the count);
    the CJK Extension I / 16.0 script ranges are already cut."""
    T = tables()
    every = set().union(*(T[n] for n in T if len(n) == 2 and n[0] in "CLMNPSZ"))
    new = [c for c in every if unicodedata.category(chr(c)) == "Cn"]
    # 14.0 added 838 code points and 15.0 4489; at most 378 more are the
    # post-15.0 remainder DESIGN.md records as a known divergence from Go 1.22
    assert len(new) <= 838 + 4489 + 378, len(new)
    assert not any(0x2EBF0 <= c <= 0x2EE5D for c in new)  # CJK Extension I (15.1)
