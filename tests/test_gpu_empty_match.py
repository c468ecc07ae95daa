"""Empty-match iteration and dense-firing custom rules.

Go's FindAllIndex / FindAllSubmatchIndex (scanner.go:107,125, regexp.go
allMatches) deliver empty matches -- stepping one rune after each, and
dropping an empty match that abuts the previous match -- and Scan emits the
span of a `secret` group even when that span is empty (scanner.go:150-163).
The engine sends rules that can match empty text to anchor-less full-file
jobs; these tests compare that path, through the C ABI, with the oracle's
restatement of Go's iteration:

* every seeded fuzz pattern (tests/test_regex_fuzz.py's generator, seed 777,
  400 cases) that can match the empty string or fires more than 12 times on
  one of its texts, as a path-scoped custom rule -- only case 354 is left
  out, by id: the oracle's backtracker (the `regex` module) goes exponential
  on it;
* hand-written empty-matching rules (`x*`, `(a|)`, `\\b`, `(?m)^`, `$`, ...);
* a `(?P<secret>[a-z]*)=` rule whose group is empty at byte 0 of the batch,
  inside a file and on the last byte of a file.

The CPU test runs the same patterns through the host Go-regexp VM
(tsg_regex_find_all) against the oracle."""
import pytest

from oracle import secret_oracle as o

from .test_regex_fuzz import _cases

N = pytest.importorskip("trivy_amd._native")

_EXPONENTIAL = {354}  # the oracle's backtracker does not finish on case 354 of seed 777

HAND = [
    r"x*", r"(a|)", r"\b", r"(?m)^", r"$", r"(?m)$", r"a*?", r"\B", r"[a-z]*", r"(?i)k*", r"^", r".*",
    r"(?s).*", r"(?:)", r"a??", r"(a*)*", r"(?m)^\s*", r"\d*", r"(?i)(key|)", r"z{0,2}", r"[^\n]*$",
    r"(?m)^[a-z]*$", r"\b\w*\b", r"(?i)\bk?e?y?", r"=*", r"(?U)a*b*", r"(|x)y?", r"[[:digit:]]*",
    r"(?m)(^|=)", r"(?s)a?.??",
]


def _selected():
    out = []
    for i, (pat, g, texts) in enumerate(_cases(777, 400)):
        if i in _EXPONENTIAL:
            continue
        if g.match_string(b"") or any(len(g.find_all_index(t)) > 12 for t in texts):
            out.append((pat, g, texts))
    return out


def _hand_texts():
    return [b"", b"a", b"key=abc\n\nxx x", b"=\n=\n", b"KEY key Key\nzz9 = a\n", b"\xc3\xa9x\xe2\x84\xaay",
            b"aaa\n\n\nbbb\n", b"x" * 70 + b"\n" + b"a b c", b"\n"]


def test_empty_and_dense_patterns_host_vm_vs_oracle():
    sel = _selected()
    assert len(sel) >= 100
    n = 0
    for pat, g, texts in sel:
        for t in texts:
            assert N.regex_find_all(pat, t) == g.find_all_index(t), (pat, t)
            n += 1
    for pat in HAND:
        g = o.GoRegexp(pat)
        for t in _hand_texts():
            assert N.regex_find_all(pat, t) == g.find_all_index(t), (pat, t)
    assert n >= 600


def _run(rules, files):
    import trivy_amd.secret as S

    from .test_gpu_parity import _canon, _oracle_plain, _plain

    cfg = S.Config(enable_builtin_rule_ids=["__none__"], custom_rules=rules)
    sc = S.new_scanner(cfg, device=0)
    oracle = o.Scanner(None)
    oracle.rules = [o.Rule(id=r.id, category=r.category, title=r.title, severity=r.severity,
                           regex=o.GoRegexp(r.regex), keywords=r.keywords, secret_group_name=r.secret_group_name,
                           path=o.GoRegexp(r.path) if r.path else None) for r in rules]
    got = sc.scan_batch([S.ScanArgs(p, d) for p, d in files])
    n = empty = 0
    for (p, d), g in zip(files, got):
        want = oracle.scan(p, d, with_offsets=True)
        n += len(want["Findings"])
        empty += sum(f.Start == f.End for f in want["Findings"])
        assert _canon(_plain(g)) == _canon(_oracle_plain(want)), p
    return n, empty


@pytest.mark.gpu
def test_empty_and_dense_fuzz_rules_on_gpu():
    import trivy_amd.secret as S

    sel = _selected()
    hand = [(pat, o.GoRegexp(pat), _hand_texts()) for pat in HAND]
    cases = sel + hand
    rules = [S.Rule(id=f"em-{i:03d}", category="Fuzz", title="empty", severity="HIGH", regex=pat,
                    path=r"^src/e%04d\.txt$" % i,
                    keywords=[] if i % 4 else [next((c for c in pat if c.isalpha()), "a")])
             for i, (pat, _, _) in enumerate(cases)]
    files = [(f"src/e{i:04d}.txt", b"\n".join(c[2])) for i, c in enumerate(cases)]
    n, empty = _run(rules, files)
    assert n > 2000 and empty > 1000


@pytest.mark.gpu
def test_empty_secret_group_at_batch_start_and_file_end():
    import trivy_amd.secret as S

    rules = [S.Rule(id="empty-group", category="Fuzz", title="empty group", severity="HIGH",
                    regex=r"(?P<secret>[a-z]*)=", secret_group_name="secret"),
             S.Rule(id="empty-x", category="Fuzz", title="x star group", severity="LOW",
                    regex=r"k(?P<secret>\d*)", secret_group_name="secret", keywords=["k"])]
    files = [
        ("a/first.txt", b"=abc\nkey=\n="),          # group empty at byte 0 of the batch and at the file's end
        ("a/mid.txt", b"x\n==\nabc=def\nk\nk12\n"),
        ("a/none.txt", b"no equals sign here\n"),
        ("a/end.txt", b"tail line\nvalue ="),        # empty group on the last byte
        ("a/only.txt", b"="),
        ("a/empty.txt", b""),
        ("a/k.txt", b"k"),
    ]
    n, empty = _run(rules, files)
    assert n >= 12 and empty >= 6
