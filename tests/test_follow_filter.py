"""Candidate filter soundness (follow.cpp, host build of the same tables the
GPU's k_expand walks): every match the Go-semantics VM finds must contain an
anchor-literal occurrence the filter accepts, else the filter would drop a
real finding.  CPU only (tsg_ruleset_follow_check runs on the host)."""
import ctypes
import os
import random

from trivy_amd import _native as N
import trivy_amd.secret as S

from . import corpus_gen
from .conftest import GOLDEN


def _rule_literals(rs, i):
    m, a, b, k = ctypes.c_int(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_size_t()
    N.check(N.lib.tsg_ruleset_rule_info(rs, i, ctypes.byref(m), ctypes.byref(a), ctypes.byref(b), ctypes.byref(k)))
    lits = []
    for j in range(k.value):
        lo, rq, ln = ctypes.create_string_buffer(256), ctypes.create_string_buffer(256), ctypes.c_size_t()
        N.check(N.lib.tsg_ruleset_rule_literal(rs, i, j, lo, rq, 256, ctypes.byref(ln)))
        lits.append((lo.raw[:ln.value], rq.raw[:ln.value]))
    return m.value, lits


def _texts():
    files = [d for _, d in corpus_gen.make_corpus(7, 80)]
    files += [open(os.path.join(GOLDEN, "secret_testdata", c), "rb").read()
              for c in sorted(os.listdir(os.path.join(GOLDEN, "secret_testdata"))) if not c.endswith(".yaml")]
    rng = random.Random(11)
    # dense adversarial texts: secrets glued together / separated by one byte
    tpl = corpus_gen.secret_instances(rng)
    for _ in range(120):
        parts = [tpl[rng.randrange(len(tpl))]() for _ in range(8)]
        files.append(rng.choice(["", " ", "\n", "'", "="]).join(parts).encode())
    return files


def test_follow_filter_never_drops_a_match():
    sc = S.new_scanner(None)
    rs = sc._rs.handle
    acc, ns = ctypes.c_int(), ctypes.c_uint32()
    texts = _texts()
    checked = filtered_rules = 0
    for i, r in enumerate(sc.rules):
        mode, lits = _rule_literals(rs, i)
        N.check(N.lib.tsg_ruleset_follow_check(rs, i, b"", 0, 0, ctypes.byref(acc), ctypes.byref(ns)))
        if mode != 1 or ns.value == 0:
            continue
        filtered_rules += 1
        for t in texts:
            low = t.lower()
            for s, e in N.regex_find_all(r.regex, t):
                ok = False
                for lo, rq in lits:
                    h = low.find(lo, s)
                    while 0 <= h and h + len(lo) <= e and not ok:
                        if all(q == 0 or t[h + k] == q for k, q in enumerate(rq)):
                            N.check(N.lib.tsg_ruleset_follow_check(rs, i, t, len(t), h, ctypes.byref(acc),
                                                                   ctypes.byref(ns)))
                            ok = acc.value == 1
                        h = low.find(lo, h + 1)
                    if ok:
                        break
                assert ok, (r.id, t[s:e])
                checked += 1
    assert filtered_rules > 70 and checked > 200


def test_follow_filter_rejects_noise():
    sc = S.new_scanner(None)
    rs = sc._rs.handle
    i = [r.id for r in sc.rules].index("twilio-api-key")
    acc, ns = ctypes.c_int(), ctypes.c_uint32()
    for text, want in [(b"SKx", 0), (b"SK" + b"a" * 31, 0), (b"SK" + b"0" * 32, 1), (b"SK\xc3\xa9", 1)]:
        N.check(N.lib.tsg_ruleset_follow_check(rs, i, text, len(text), 0, ctypes.byref(acc), ctypes.byref(ns)))
        assert acc.value == want, text
