"""Verify-DFA exactness (dfa.cpp, the host build of the tables k_verify walks):
Go's FindAllIndex rebuilt from the anchored leftmost-first DFA (leftmost
start = first start position with a match, end = the DFA's match end) must
equal the host Go-semantics Pike VM's FindAllIndex on ASCII text, for every
builtin rule and a few hand-picked priority/assertion patterns.  CPU only."""
import ctypes
import os
import random

import pytest

from trivy_amd import _native as N
import trivy_amd.secret as S

from . import corpus_gen
from .conftest import GOLDEN


def _dfa_find_all(rs, i, t):
    res, me, ns = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_uint32()
    out, pos, n = [], 0, len(t)
    while pos < n:
        hit = None
        for s in range(pos, n):
            N.check(N.lib.tsg_ruleset_dfa_check(rs, i, t, n, s, ctypes.byref(res), ctypes.byref(me), ctypes.byref(ns)))
            assert res.value != 2, "ASCII text must be decidable"
            if res.value == 1:
                hit = (s, me.value)
                break
        if hit is None:
            break
        assert hit[1] > hit[0], "anchored builtin rules never match empty"
        out.append(list(hit))
        pos = hit[1]
    return out


def _ascii_texts():
    rng = random.Random(5)
    tpl = corpus_gen.secret_instances(rng)
    texts = [d for _, d in corpus_gen.make_corpus(3, 40) if max(d, default=0) < 0x80]
    texts += [open(os.path.join(GOLDEN, "secret_testdata", c), "rb").read()
              for c in sorted(os.listdir(os.path.join(GOLDEN, "secret_testdata"))) if not c.endswith(".yaml")]
    texts = [t for t in texts if max(t, default=0) < 0x80 and len(t) < 6000]
    for _ in range(60):
        parts = [tpl[rng.randrange(len(tpl))]() for _ in range(5)]
        t = rng.choice(["", " ", "\n", "'", "=", "\t\n  "]).join(parts).encode()
        if max(t, default=0) < 0x80:
            texts.append(t)
    return texts


def test_verify_dfa_equals_vm_on_builtin_rules():
    sc = S.new_scanner(None)
    rs = sc._rs.handle
    res, me, ns = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_uint32()
    texts = _ascii_texts()
    total = 0
    for i, r in enumerate(sc.rules):
        N.check(N.lib.tsg_ruleset_dfa_check(rs, i, b"x", 1, 0, ctypes.byref(res), ctypes.byref(me), ctypes.byref(ns)))
        if ns.value == 0:
            continue
        for t in texts:
            want = N.regex_find_all(r.regex, t)
            if not want and r.keywords and not any(k.lower().encode() in t.lower() for k in r.keywords):
                continue  # keep the O(n^2) reference walk to texts that matter
            assert _dfa_find_all(rs, i, t) == want, (r.id, t[:120])
            total += len(want)
    assert total > 200


@pytest.mark.parametrize("pat,text", [
    (r"(a|ab)(c|bcd)(d*)", b"abcd xabcdd"), (r"x*?y", b"xxy xy"), (r"a+?", b"aaa"), (r"(?U)a+", b"aaa b"),
    (r"^abc", b"abc abc"), (r"abc$", b"abc abc"), (r"(^|\s+)k(\s+|$)", b"k  k \n k"), (r"a{2,3}", b"aaaaaaa"),
    (r"(?i)key[a-z]{0,3}=", b"KEYab= keyabcd="), (r"([^0-9A-Za-z]|^)(LTAI)(?i)[a-z0-9]{4}([^0-9A-Za-z]|$)", b"LTAIabcd xLTAI1234 LTAIzzzz"),
])
def test_verify_dfa_priorities(pat, text):
    rules = [S.Rule(id="t", category="c", title="t", severity="HIGH", regex=pat, keywords=[])]
    sc = S.Scanner(rules, [], S.ExcludeBlock())
    rs = sc._rs.handle
    res, me, ns = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_uint32()
    N.check(N.lib.tsg_ruleset_dfa_check(rs, 0, b"x", 1, 0, ctypes.byref(res), ctypes.byref(me), ctypes.byref(ns)))
    if ns.value == 0:
        pytest.skip("no DFA for this pattern (VM path)")
    assert _dfa_find_all(rs, 0, text) == N.regex_find_all(pat, text)


def _rune_starts(t: bytes):
    """Byte offsets where utf8.DecodeRune starts a rune (invalid byte = width 1)."""
    s = t.decode("utf-8", "surrogateescape")
    out, b = [], 0
    for ch in s:
        out.append(b)
        cp = ord(ch)
        b += 1 if (0xDC80 <= cp <= 0xDCFF or cp < 0x80) else 2 if cp < 0x800 else 3 if cp < 0x10000 else 4
    return out


def _dfa_find_all_runes(rs, i, t):
    """FindAllIndex from the DFA over rune starts; None if some start is left to the VM."""
    res, me, ns = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_uint32()
    starts = _rune_starts(t)
    out, pos = [], 0
    while True:
        hit = None
        for s in starts:
            if s < pos:
                continue
            N.check(N.lib.tsg_ruleset_dfa_check(rs, i, t, len(t), s, ctypes.byref(res), ctypes.byref(me), ctypes.byref(ns)))
            if res.value == 2:
                return None
            if res.value == 1:
                hit = (s, me.value)
                break
        if hit is None:
            return out
        out.append(list(hit))
        pos = hit[1]


def test_verify_dfa_rune_symbols_equal_vm():
    """Non-ASCII text: the DFA's rune symbols (K, ſ, İ, U+FFFD, other runes)
    give the VM's matches, for every builtin rule whose classes treat other
    non-ASCII runes alike (the device leaves the rest to the VM)."""
    rng = random.Random(17)
    tpl = corpus_gen.secret_instances(rng)
    fold = {"k": "K", "K": "K", "s": "ſ", "S": "ſ", "i": "İ"}
    texts = []
    for _ in range(120):
        parts = []
        for _ in range(3):
            x = tpl[rng.randrange(len(tpl))]()
            x = "".join(fold[c] if c in fold and rng.random() < 0.3 else c for c in x)
            parts.append(x)
        t = rng.choice([" é ", "\n", "'ſ'", " ÿ "]).join(parts).encode()
        if rng.random() < 0.3:
            p = rng.randrange(len(t) + 1)
            t = t[:p] + bytes([rng.randint(0x80, 0xFF)]) + t[p:]
        texts.append(t)
    sc = S.new_scanner(None)
    rs = sc._rs.handle
    res, me, ns = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_uint32()
    decided = total = 0
    for i, r in enumerate(sc.rules):
        N.check(N.lib.tsg_ruleset_dfa_check(rs, i, b"x", 1, 0, ctypes.byref(res), ctypes.byref(me), ctypes.byref(ns)))
        if ns.value == 0:
            continue
        for t in texts:
            got = _dfa_find_all_runes(rs, i, t)
            if got is None:
                continue
            want = N.regex_find_all(r.regex, t)
            assert got == want, (r.id, t[:160])
            decided += 1
            total += len(want)
    assert decided > 5000 and total > 100


def test_accelerated_walk_equals_plain_walk():
    """k_verify's run acceleration (engine.hip dfa_accel_skip: a state whose
    entry is the same on all but <= 3 ASCII bytes skips runs of the others
    with vector compares), restated on the host, gives the plain walk's
    answer from every start of ASCII, non-ASCII and private-key texts, for
    every builtin rule with a verify DFA; the private-key body is skipped."""
    sc = S.new_scanner(None)
    rs = sc._rs.handle
    rng = random.Random(17)
    texts = _ascii_texts()[:40]
    body = "".join(rng.choice("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/\n") for _ in range(3000))
    key = ("-----BEGIN RSA PRIVATE KEY-----\n" + body + "\n-----END RSA PRIVATE KEY-----\n").encode()
    texts += [key, key[:-5], b"x = " + key + b" tail", "é ſ K ".encode() + key, key.replace(b"Q", "é".encode())]
    res, me, ns = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_uint32()
    ares, ame, sk = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_uint64()
    skipped = checked = 0
    for i in range(N.lib.tsg_ruleset_rule_count(rs)):
        N.check(N.lib.tsg_ruleset_dfa_check(rs, i, b"x", 1, 0, ctypes.byref(res), ctypes.byref(me), ctypes.byref(ns)))
        if not ns.value:
            continue
        for t in texts:
            starts = range(len(t)) if len(t) < 400 else sorted(rng.sample(range(len(t)), 150) + [0, len(t) - 1])
            for s in starts:
                N.check(N.lib.tsg_ruleset_dfa_check(rs, i, t, len(t), s, ctypes.byref(res), ctypes.byref(me),
                                                    ctypes.byref(ns)))
                N.check(N.lib.tsg_ruleset_dfa_accel_check(rs, i, t, len(t), s, ctypes.byref(ares), ctypes.byref(ame),
                                                          ctypes.byref(sk)))
                assert ares.value == res.value and (res.value != 1 or ame.value == me.value), (i, s)
                skipped += sk.value
                checked += 1
    assert checked > 10000 and skipped > 5000
    pk = next(i for i in range(N.lib.tsg_ruleset_rule_count(rs)) if sc.rules[i].id == "private-key")
    N.check(N.lib.tsg_ruleset_dfa_accel_check(rs, pk, key, len(key), 0, ctypes.byref(ares), ctypes.byref(ame),
                                              ctypes.byref(sk)))
    assert ares.value == 1 and ame.value == len(key) - 1 and sk.value > 2900  # the body: runs of base64 bytes
