"""Scan-automaton class extensions (ruleset.cpp build_fast, follow.cpp
follow_ext): k_scan_fast only reports an anchor literal when the next `ext`
bytes fold into the column sets the rule requires there.  Soundness: every
match the Go-semantics VM finds must contain an occurrence of one of its
rule's anchor literals whose following bytes pass those sets (the anchor hit
that lets k_verify find the match).  CPU only (host tables)."""
import ctypes

from trivy_amd import _native as N
import trivy_amd.secret as S

from .test_follow_filter import _rule_literals, _texts


def _fold(b):
    return (b & 0x1F) | ((b >> 1) & 0x20)


def _scan_patterns(rs):
    st = [ctypes.c_uint32() for _ in range(4)]
    fp = ctypes.c_int()
    N.check(N.lib.tsg_ruleset_stats(rs, *[ctypes.byref(x) for x in st], ctypes.byref(fp)))
    out = {}
    states = 0
    for k in range(st[2].value):
        buf, n, e = ctypes.create_string_buffer(256), ctypes.c_size_t(), ctypes.c_uint32()
        cols, fs = (ctypes.c_uint64 * 8)(), ctypes.c_uint32()
        N.check(N.lib.tsg_ruleset_scan_pattern(rs, k, buf, 256, ctypes.byref(n), ctypes.byref(e), cols,
                                               ctypes.byref(fs)))
        out[buf.raw[:n.value]] = [cols[j] for j in range(e.value)]
        states = fs.value
    return out, states, fp.value


def _passes(t, h, n, cols):
    for j, m in enumerate(cols):
        q = h + n + j
        if q >= len(t) or not (m >> _fold(t[q])) & 1:
            return False
    return True


def test_extensions_present_and_fit():
    sc = S.new_scanner(None)
    pats, states, fast = _scan_patterns(sc._rs.handle)
    assert fast == 1 and 0 < states <= 1008
    # the frequent short literals carry classes (twilio's SK + hex digits)
    assert len(pats[b"sk"]) >= 2
    hexcols = {_fold(c) for c in b"0123456789abcdefABCDEF"}
    assert all({v for v in range(64) if (m >> v) & 1} == hexcols for m in pats[b"sk"])


def test_extensions_never_drop_a_match():
    sc = S.new_scanner(None)
    rs = sc._rs.handle
    pats, _, _ = _scan_patterns(rs)
    texts = _texts()
    checked = extended = 0
    for i, r in enumerate(sc.rules):
        mode, lits = _rule_literals(rs, i)
        if mode != 1 or not any(pats.get(lo) for lo, _ in lits):
            continue
        extended += 1
        for t in texts:
            low = t.lower()
            for s, e in N.regex_find_all(r.regex, t):
                ok = False
                for lo, rq in lits:
                    h = low.find(lo, s)
                    while 0 <= h and h + len(lo) <= e and not ok:
                        if all(q == 0 or t[h + k] == q for k, q in enumerate(rq)):
                            ok = _passes(t, h, len(lo), pats.get(lo, []))
                        h = low.find(lo, h + 1)
                    if ok:
                        break
                assert ok, (r.id, t[s:e])
                checked += 1
    assert extended >= 5 and checked > 50


def test_extensions_reject_noise():
    sc = S.new_scanner(None)
    pats, _, _ = _scan_patterns(sc._rs.handle)
    cols = pats[b"sk"]
    assert not _passes(b"task runner", 2, 2, cols)
    assert _passes(b"SK0123abcd", 0, 2, cols)
