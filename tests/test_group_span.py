"""Secret-group spans from the match span alone (gre::group_span, used by
k_verify's emit_match to skip the capture search): for every rule the
analysis accepts, the group of every ASCII match must equal the oracle's
FindAllSubmatchIndex group (getMatchSubgroupsLocations, scanner.go:150-163),
and the analysis must refuse groups that can be absent, repeat, or sit
between variable-length parts.  CPU only (host ABI + oracle)."""
import ctypes
import random

import pytest

from oracle import secret_oracle as O
from tests import corpus_gen

N = pytest.importorskip("trivy_amd._native")
S = pytest.importorskip("trivy_amd.secret")


def _span(sc, i):
    v = [ctypes.c_int() for _ in range(4)]
    N.check(N.lib.tsg_ruleset_group_span(sc._rs.handle, i, *[ctypes.byref(x) for x in v]))
    return [x.value for x in v]


def _derive(sp, ms, me):
    valid, pre, ln, suf = sp
    gs = ms + pre if pre >= 0 else me - suf - ln
    ge = me - suf if suf >= 0 else gs + ln
    return gs, ge


def _gen_files(seed, n_files, size=1 << 16, density=2e-3):
    """Files of the bench corpus generator (corpus.hip: every builtin rule's
    template planted round-robin), at a high plant density."""
    out = []
    for f in range(n_files):
        buf = ctypes.create_string_buffer(size)
        N.check(N.gen.tsg_gen_file(seed, f, size, density, buf))
        out.append(buf.raw)
    return out


def _texts(seed):
    rng = random.Random(seed)
    out = [d for _, d in corpus_gen.make_corpus(seed, 120)] + _gen_files(seed, 64)
    # adversarial: quote runs, repeated keys, long separators
    for _ in range(200):
        inst = corpus_gen.secret_instances(rng)
        line = rng.choice(inst)()
        pad = rng.choice(['"', "'", " ", "=", ":", '""', "x" * rng.randint(0, 30)])
        out.append((pad + line + pad + rng.choice(['"', "'", "\n", ""]) + line).encode("utf-8", "surrogateescape"))
    return out


def test_builtin_group_spans_equal_oracle_captures():
    sc = S.new_scanner(None)
    texts = _texts(4242)
    accepted, checked, seen = 0, 0, set()
    for i, r in enumerate(sc.rules):
        if not r.secret_group_name:
            continue
        sp = _span(sc, i)
        if not sp[0]:
            continue
        accepted += 1
        rx = O.GoRegexp(r.regex)
        names = rx.subexp_names()
        g = names.index(r.secret_group_name)
        for t in texts:
            for m in rx.find_all_submatch_index(t):
                ms, me = m[0], m[1]
                if any(b >= 0x80 for b in t[ms:me]):
                    continue
                assert (m[2 * g], m[2 * g + 1]) == _derive(sp, ms, me), (r.id, t[ms:me])
                checked += 1
                seen.add(r.id)
    assert accepted >= 30 and checked >= 1500, (accepted, checked)
    assert len(seen) == accepted, sorted(set(r.id for r in sc.rules if r.secret_group_name) - seen)


@pytest.mark.parametrize("regex,want", [
    (r"x(?P<secret>[a-z]+)y", [1, 1, -1, 1]),
    (r"a.{0,5}(?P<secret>b{3})", [1, -1, 3, 0]),
    (r"(?P<secret>[0-9]{4})[a-z]*", [1, 0, 4, -1]),
    (r"(?P<secret>a){2}", [0, -1, -1, -1]),          # the group repeats
    (r"c|(?P<secret>b)", [0, -1, -1, -1]),           # the group may not participate
    (r"(?P<secret>b)?", [0, -1, -1, -1]),
    (r"[a-z]+(?P<secret>[0-9]+)[a-z]+", [0, -1, -1, -1]),  # variable on every side
    (r"(?i)k(?P<secret>[a-z]{2})s", [1, 1, 2, 1]),   # rune counts: applied to ASCII matches only
])
def test_group_span_analysis(regex, want):
    cfg = S.Config(enable_builtin_rule_ids=["__none__"],
                   custom_rules=[S.Rule(id="r", regex=regex, keywords=[], secret_group_name="secret")])
    sc = S.new_scanner(cfg)
    assert len(sc.rules) == 1
    assert _span(sc, 0) == want
    if want[0]:
        rx = O.GoRegexp(regex)
        rng = random.Random(1)
        for _ in range(300):
            t = "".join(rng.choice("abcxy0123 ks") for _ in range(rng.randint(0, 40))).encode()
            for m in rx.find_all_submatch_index(t):
                assert (m[2], m[3]) == _derive(want, m[0], m[1])


# --- byte runs (gre::group_run): groups between variable-length parts --------

def _run_rule(sc, i):
    v, ln = ctypes.c_int(), ctypes.c_int()
    sa = (ctypes.c_uint32 * 4)()
    ba = (ctypes.c_uint32 * 4)()
    N.check(N.lib.tsg_ruleset_group_run(sc._rs.handle, i, ctypes.byref(v), ctypes.byref(ln), sa, ba))
    return v.value, list(sa), list(ba), ln.value


def _derive_run(rr, t, ms, me):
    _, sa, ba, ln = rr
    inn = lambda m, c: (m[c >> 5] >> (c & 31)) & 1  # noqa: E731
    ge = me
    while ge > ms and inn(sa, t[ge - 1]):
        ge -= 1
    if ln >= 0:
        return ge - ln, ge
    gs = ge
    while gs > ms and inn(ba, t[gs - 1]):
        gs -= 1
    return gs, ge


def _check_run_rules(sc, texts, min_checked):
    accepted, checked, seen = 0, 0, set()
    for i, r in enumerate(sc.rules):
        if not r.secret_group_name or _span(sc, i)[0]:
            continue
        rr = _run_rule(sc, i)
        if not rr[0]:
            continue
        accepted += 1
        rx = O.GoRegexp(r.regex)
        g = rx.subexp_names().index(r.secret_group_name)
        for t in texts:
            for m in rx.find_all_submatch_index(t):
                ms, me = m[0], m[1]
                if any(b >= 0x80 for b in t[ms:me]):
                    continue
                assert (m[2 * g], m[2 * g + 1]) == _derive_run(rr, t, ms, me), (r.id, t[ms:me])
                checked += 1
                seen.add(r.id)
    assert checked >= min_checked, (accepted, checked)
    return accepted, seen


def test_builtin_group_runs_equal_oracle_captures():
    """aws-secret-access-key (an optional quote, [.,] and a whitespace run
    after the secret) and every other builtin group rule the span shortcut
    refuses but the run analysis accepts."""
    sc = S.new_scanner(None)
    accepted, seen = _check_run_rules(sc, _texts(777), 50)
    assert "aws-secret-access-key" in seen
    assert len(seen) == accepted


def test_stress_group_runs_equal_oracle_captures():
    """The configs[4] gitleaks-shaped rules: keyword, separator class {0,20},
    quote runs, operator, quote-or-space {0,5}, the secret, a terminator or $."""
    from tests import stress_rules
    rules = stress_rules.make_rules(20261019, 120)
    custom = [S.Rule(id=r["id"], regex=r["regex"], keywords=r.get("keywords", []),
                     secret_group_name=r.get("secret-group-name", "")) for r, _ in rules]
    sc = S.new_scanner(S.Config(enable_builtin_rule_ids=["__none__"], custom_rules=custom))
    rng = random.Random(5)
    texts = []
    gens = [g for _, g in rules if g is not None]
    for _ in range(300):
        parts = [rng.choice(gens)(rng) for _ in range(rng.randint(1, 6))]
        texts.append((rng.choice(["", " ", "\n", "x=", "'"]).join(parts) + rng.choice(["", "\n", " ", ";"])).encode())
    accepted, seen = _check_run_rules(sc, texts, 300)
    fam = [r["id"] for i, (r, _) in enumerate(rules) if i % 10 in (0, 1, 2, 3)]
    assert accepted >= len(fam) * 0.9, (accepted, len(fam))


@pytest.mark.parametrize("regex,valid", [
    (r"k[a-z ]{0,5}=\s*['\"]?(?P<secret>[0-9a-f]{8,40})['\"]?(\s|$)", 1),
    (r"k *=(?P<secret>[0-9a-z]+)[a-z]*", 0),        # the tail can eat the secret's bytes
    (r"k[0-9]*(?P<secret>[0-9]+)x+", 0),            # the head can end in the secret's bytes
    (r"k *=(?P<secret>[0-9]*)x+", 0),               # the group may be empty
    (r"k *=(?P<secret>[0-9a-f]{12})['\"]?;*", 1),   # fixed length: only the end needs the runs
    (r"(?:k=(?P<secret>[0-9]+);)+", 0),             # the group repeats
])
def test_group_run_analysis(regex, valid):
    cfg = S.Config(enable_builtin_rule_ids=["__none__"],
                   custom_rules=[S.Rule(id="r", regex=regex, keywords=[], secret_group_name="secret")])
    sc = S.new_scanner(cfg)
    assert _span(sc, 0)[0] == 0
    rr = _run_rule(sc, 0)
    assert rr[0] == valid
    if valid:
        rx = O.GoRegexp(regex)
        rng = random.Random(2)
        for _ in range(400):
            t = "".join(rng.choice("k= '\"0123abcf9x") for _ in range(rng.randint(0, 60))).encode()
            for m in rx.find_all_submatch_index(t):
                assert (m[2], m[3]) == _derive_run(rr, t, m[0], m[1])
