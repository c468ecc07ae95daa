"""Go regexp Unicode classes: \\pN, \\p{Name}, \\P{Name}, \\p{^Name}
(regexp/syntax parse.go parseUnicodeClass / unicodeTable) in gre.cpp.

* Known answers for the Go 1.22 tables (oracle/go_unicode.py, Unicode 15.0):
  code points whose category / script Go's `unicode` package fixes.
* The host compiler + VM (tsg_regex_find_all) against the oracle on patterns
  mixing classes, negation, (?i) fold closure and bracket classes.
* Compile errors: an unknown name is Go's "invalid character class range"
  (TSG_ERR_REGEX, "regexp compile error" at config decode); a feature outside
  this engine's coverage (a keyword with invalid UTF-8) is TSG_ERR_UNSUPPORTED (5).
* GPU: custom rules with \\p{L} and \\p{Greek} through the C-ABI scan, findings
  compared field by field with the oracle Scanner.
"""
import ctypes
import random

import pytest

from oracle import go_unicode as U
from oracle import secret_oracle as o

N = pytest.importorskip("trivy_amd._native")
S = pytest.importorskip("trivy_amd.secret")


def _has(name, cp):
    return cp in U.table(name)


def test_known_answers():
    assert _has("Lu", ord("A")) and _has("L", ord("z")) and not _has("L", ord("1"))
    assert _has("Lt", 0x01C5)                         # ǅ titlecase
    assert _has("Greek", ord("α")) and _has("Greek", 0x2126)  # Ω OHM SIGN is Greek script
    assert _has("Common", 0x00B5) and _has("Ll", 0x00B5)       # µ MICRO SIGN
    assert _has("Han", ord("中")) and _has("Nd", ord("٣"))
    assert _has("Kawi", 0x11F00) and _has("Nag_Mundari", 0x1E4D0)  # 15.0 scripts
    assert _has("Vithkuqi", 0x10570)                                # 14.0
    assert not _has("Egyptian_Hieroglyphs", 0x13460)  # Extended-A is 16.0: unassigned in Go 1.22
    assert not _has("L", 0x10D50)                     # Garay (16.0)
    assert not _has("Han", 0x2EBF0)                   # CJK Extension I (15.1)
    assert _has("C", 0x0000) and _has("C", 0xE000) and _has("C", 0xD800)  # Cc, Co, Cs
    assert not _has("C", 0x0378)                       # unassigned: in no Go table
    assert U.table("Foo") is None and U.table("Unknown") is None and U.table("LC") is None
    # (?i) fold additions (FoldScript / FoldCategory)
    assert 0x00B5 in U.fold_closure("Greek")            # µ joins Greek via the Μ/μ orbit
    assert 0x0345 in U.fold_closure("Greek") or _has("Inherited", 0x0345)
    assert ord("k") in U.fold_closure("Lu") and 0x212A in U.fold_closure("Ll")
    assert 0x0130 not in U.fold_closure("Ll")           # İ stays out of the i orbit


_PATTERNS = [
    r"\pL+", r"\p{L}+", r"\PL+", r"\P{L}{2,}", r"\p{^L}+", r"\P{^Greek}+", r"\p{Greek}+", r"\p{Lu}\p{Ll}+",
    r"(?i)\p{Lu}+", r"(?i)\P{Lu}+", r"(?i)\p{Greek}+", r"[\p{Nd}x]+", r"[^\p{L}\s]+", r"(?i)[^\p{Lu}k]+",
    r"[\p{Han}\p{Hiragana}]+", r"\p{Any}{3}", r"\pN\pP", r"[\p{Cyrillic}-]+", r"\p{Zs}", r"\p{Sc}\d+",
    r"\p{Common}+", r"\p{Inherited}", r"\p{Cc}+", r"\p{So}",
]

_TEXTS = [
    "Ωmega αβγ µ ΜΙΚΡΟ δ3 Kelvin K ſharp İstanbul ıi".encode(),
    "Привет-мир 中文テキスト ひらがな 123 ٣٤ €42 ¥7 ǅemal ǆ Ǆ".encode(),
    b"plain ascii 42, fine!\t\x01\x7f",
    b"bad \xff\xfe utf8 \xc3 \xe2\x82 tail",
    "e\u0301 combining \u0345 ypogegrammeni 𝐀𝐁 𝟘 emoji 😀 \u00a0nbsp".encode(),
]


@pytest.mark.parametrize("pat", _PATTERNS)
def test_host_vm_unicode_classes_vs_oracle(pat):
    g = o.GoRegexp(pat)
    for t in _TEXTS:
        assert N.regex_find_all(pat, t) == g.find_all_index(t), (pat, t)


def test_host_vm_unicode_random_runes():
    rng = random.Random(20261016)
    pool = [c for c in range(0x80, 0x30000) if not 0xD800 <= c <= 0xDFFF]
    for pat in [r"\p{L}+", r"(?i)\p{Lu}", r"\P{Greek}\p{Greek}", r"[\p{Nd}\p{Nl}]+", r"\p{M}"]:
        g = o.GoRegexp(pat)
        for _ in range(6):
            t = "".join(chr(rng.choice(pool)) if rng.random() < 0.7 else rng.choice("aZ9 -K")
                        for _ in range(300)).encode("utf-8", "surrogatepass")
            assert N.regex_find_all(pat, t) == g.find_all_index(t), pat


@pytest.mark.parametrize("bad,expr", [(r"\p{Foo}", r"\p{Foo}"), (r"a\pX", r"\pX"), (r"[\P{Bar}]", r"\P{Bar}"),
                                      (r"\p{L", r"\p{L"), (r"x\p", r"\p"), (r"\p{LC}", r"\p{LC}")])
def test_unknown_class_is_go_compile_error(bad, expr):
    m = ctypes.c_int()
    rc = N.lib.tsg_regex_match(bad.encode(), b"", 0, ctypes.byref(m))
    assert rc == N.TSG_ERR_REGEX
    msg = N.lib.tsg_last_error().decode()
    assert "invalid character class range" in msg and ("`%s`" % expr) in msg, msg
    with pytest.raises(o.GoSyntaxError):
        o.GoRegexp(bad)


def test_outside_coverage_is_unsupported():
    # a keyword with invalid UTF-8 (Go would lower it through RuneError)
    bad = S.Rule(id="bad-kw", category="c", title="t", severity="HIGH", regex="x", keywords=["cl\udce9"])
    with pytest.raises(N.EngineError) as ei:
        S.new_scanner(S.Config(custom_rules=[bad]))
    assert ei.value.code == N.TSG_ERR_UNSUPPORTED


_CFG = r"""
rules:
  - id: letters-token
    category: test
    title: token of letters
    severity: HIGH
    regex: 'token=(?P<secret>\p{L}{6,})'
    secret-group-name: secret
    keywords: [token=]
  - id: greek-key
    category: test
    title: greek key
    severity: MEDIUM
    regex: 'greek:\s*\p{Greek}{4,}'
    keywords: [greek]
  - id: not-letters
    category: test
    title: non-letters then upper
    severity: LOW
    regex: '(?i)pass=[\P{L}]{4}\p{Lu}'
    keywords: [pass=]
  - id: caret-digits
    category: test
    title: caret class
    severity: LOW
    regex: 'sym=\p{^Nd}{3}\pN+'
  - id: greek-full
    category: test
    title: keyword-less greek digits
    severity: LOW
    regex: '\p{Greek}{3}\d{4}'
"""


def _files():
    rng = random.Random(7)
    greek = "αβγδεζηθικλμνξοπρστυφχψω"
    lines = [
        "token=Ωmegaλόγος ok", "token=abcdefg", "token=ab12", "token=Привет12", "greek: αβγδε and more",
        "greek:ΑΒΓ no", "pass=1234Ä!", "PASS=!!!!Z", "pass=abcdZ", "sym=abc٣٤5", "sym=a1c99", "ωψχ2024",
        "µµµ1234", "token=ſtraßeK done", "İ token=İİİİİİ", "bad \xff bytes token=ééééééé",
    ]
    files = []
    for i in range(40):
        body = []
        for _ in range(rng.randint(5, 40)):
            r = rng.random()
            if r < 0.4:
                body.append(rng.choice(lines))
            elif r < 0.6:
                body.append("".join(rng.choice(greek) for _ in range(rng.randint(1, 12))) + str(rng.randint(0, 99999)))
            else:
                body.append("filler text %d %s" % (i, "x" * rng.randint(0, 60)))
        data = "\n".join(body).encode("utf-8", "surrogateescape")
        if i % 7 == 3:
            data = data.replace(b"\xc3\xbf", b"\xff")
        files.append(("dir/f%02d.txt" % i, data))
    return files


@pytest.mark.gpu
def test_gpu_unicode_class_rules_vs_oracle(tmp_path):
    from .test_gpu_parity import _canon, _oracle_plain, _plain
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text(_CFG)
    sc_o = o.Scanner(o.parse_config(str(cfg)))
    sc_g = S.new_scanner(S.parse_config(str(cfg)), device=0)
    files = _files()
    got = sc_g.scan_batch([S.ScanArgs(p, d) for p, d in files])
    seen = set()
    for (p, d), g in zip(files, got):
        want = _oracle_plain(sc_o.scan(p, d))
        seen |= {f["RuleID"] for f in want["Findings"]}
        assert _canon(_plain(g)) == _canon(want), p
    assert {"letters-token", "greek-key", "greek-full", "caret-digits"} <= seen
