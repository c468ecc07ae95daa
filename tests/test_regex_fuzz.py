"""Randomised Go-regexp parity: seeded random patterns
built from the RE2 syntax custom `trivy-secret.yaml` rules use (literals,
escapes, classes, POSIX classes, `.`, groups, named groups, alternation,
greedy / lazy repetition with counts, `^ $ \\b \\B`, `(?i)`, `(?s)`, `(?m)`)
against the oracle's restatement of Go's leftmost-first `FindAllIndex`
(regexp.go allMatches) on random texts biased towards matching.

CPU test: the engine's own compiler + host Pike VM through the C ABI
(tsg_regex_find_all).  The GPU test feeds the same kind of patterns as custom
rules through the whole device path (anchors, follow filter, verify DFA,
Pike VM, findings) and compares the findings with the oracle's Scan."""
import random

import pytest

from oracle import secret_oracle as o

N = pytest.importorskip("trivy_amd._native")

ALPHA = "abcxyz_-=:0129"


def _atom(rng, depth):
    k = rng.random()
    if depth > 0 and k < 0.22:
        inner = _alt(rng, depth - 1)
        return rng.choice(["(%s)", "(?:%s)", "(?P<g%d>%%s)" % rng.randrange(3)]) % inner
    if k < 0.45:
        return rng.choice(ALPHA.replace("-", "").replace("=", ""))
    if k < 0.55:
        return rng.choice([r"\d", r"\w", r"\s", r"\D", r"\W", r"\.", r"\-", r"\x61", r"\b", r"\B"])
    if k < 0.72:
        body = rng.choice(["a-c", "^a", "xyz", "0-9_", "[:digit:]", "[:alpha:]", "a-z0-9", "^\\n", "=:"])
        return "[" + body + "]"
    if k < 0.8:
        return "."
    if k < 0.84:
        return rng.choice(["^", "$"])
    return rng.choice(["ab", "xy", "key", "z="])


def _piece(rng, depth):
    a = _atom(rng, depth)
    if a in ("^", "$", r"\b", r"\B"):
        return a
    k = rng.random()
    if k < 0.5:
        return a
    rep = rng.choice(["*", "+", "?", "{2}", "{1,3}", "{0,2}", "{2,}", "*?", "+?", "??", "{1,2}?"])
    return a + rep


def _concat(rng, depth):
    return "".join(_piece(rng, depth) for _ in range(rng.randint(1, 4)))


def _alt(rng, depth):
    return "|".join(_concat(rng, depth) for _ in range(rng.randint(1, 2 if depth else 3)))


def random_pattern(rng):
    p = _alt(rng, 2)
    flags = rng.choice(["", "", "", "(?i)", "(?s)", "(?m)", "(?is)"])
    return flags + p


def random_text(rng, pat):
    # fragments of the pattern's literals make matches likely
    frags = [c for c in pat if c in ALPHA] or ["a"]
    out = []
    for _ in range(rng.randint(0, 60)):
        k = rng.random()
        if k < 0.55:
            out.append(rng.choice(frags))
        elif k < 0.85:
            out.append(rng.choice(ALPHA + "  \n"))
        elif k < 0.95:
            out.append(rng.choice(["ABC", "Key", "XY", "\t"]))
        else:
            out.append(rng.choice(["é", "K", "ſ", "K"]))
    return "".join(out).encode("utf-8")


def _cases(seed, n):
    rng = random.Random(seed)
    out = []
    while len(out) < n:
        pat = random_pattern(rng)
        try:
            g = o.GoRegexp(pat)
        except Exception:  # noqa: BLE001  (outside the oracle's translation: not a parity case)
            continue
        out.append((pat, g, [random_text(rng, pat) for _ in range(6)]))
    return out


def test_random_patterns_host_vm_vs_oracle():
    checked = matched = 0
    for pat, g, texts in _cases(20261017, 500):
        for t in texts:
            want = g.find_all_index(t)
            assert N.regex_find_all(pat, t) == want, (pat, t)
            checked += 1
            matched += bool(want)
    assert checked == 3000 and matched > 800


@pytest.mark.gpu
def test_random_patterns_as_custom_rules_on_gpu():
    import trivy_amd.secret as S

    from .test_gpu_parity import _canon, _oracle_plain, _plain

    # rules that cannot match empty text and do not fire on every other byte
    # (the first 250 seeded cases: case 354 sends the oracle's backtracker
    # exponential).  Each rule is path-scoped to its own file (Rule.Path,
    # scanner.go:165-167), so the oracle runs each pattern only on the texts
    # it was generated with; the GPU evaluates the path gates itself.
    cases = [c for c in _cases(777, 250)
             if not c[1].match_string(b"") and all(len(c[1].find_all_index(t)) <= 12 for t in c[2])][:120]
    path = [f"src/f{i:04d}.txt" for i in range(len(cases))]
    scope = [r"^src/f%04d\.txt$" % i for i in range(len(cases))]
    rules = [S.Rule(id=f"fz-{i:03d}", category="Fuzz", title="fuzz", severity="HIGH", regex=pat, path=scope[i],
                    keywords=[] if i % 3 else [next((c for c in pat if c.isalpha()), "a")])
             for i, (pat, _, _) in enumerate(cases)]
    cfg = S.Config(enable_builtin_rule_ids=["__none__"], custom_rules=rules)
    sc = S.new_scanner(cfg, device=0)
    oracle = o.Scanner(None)
    oracle.rules = [o.Rule(id=r.id, category=r.category, title=r.title, severity=r.severity,
                           regex=o.GoRegexp(r.regex), keywords=r.keywords, path=o.GoRegexp(r.path)) for r in rules]
    files = [(path[i], b"\n".join(cases[i][2])) for i in range(len(cases))]
    got = sc.scan_batch([S.ScanArgs(p, d) for p, d in files])
    n = 0
    for (p, d), g in zip(files, got):
        want = _oracle_plain(oracle.scan(p, d))
        n += len(want["Findings"])
        assert _canon(_plain(g)) == _canon(want), p
    assert n > 100
