#!/usr/bin/env python3
"""Would a VALU-only prefilter take k_scan_fast off its LDS-gather ceiling?
(CPU simulation on the bench corpus text model)

k_scan_fast walks a 1003-row fold-column DFA (one dependent ds_read_u16 per
byte).  A prefilter in front of it would let the DFA run only on flagged
8-byte groups (restarting from the 7-byte look-back).  It pays only when few
groups are flagged, so this measures the flagged-group rate of:

1. the EXACT k-prefix filter (a position is flagged iff the next k fold
   columns are a prefix of some scan pattern, class extensions included) --
   the lower bound of every prefilter that looks at k bytes;
2. Teddy / FDR-style nibble buckets (8 or 16 buckets; per position offset
   j < k two 8-entry tables indexed by column bits 0-2 and 3-5, as v_perm_b32
   lookups from VGPR-resident tables would do); patterns assigned to buckets
   greedily by the flagged positions they add;
3. a stride-2 exact 3-gram bitmap (32 KiB in LDS, half the lookups of the
   DFA, no dependent chain), priced with the same 32-lane LDS bank model as
   tools/bank_sim.py.

Usage: python tools/prefilter_sim.py [regions]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bank_sim as B  # noqa: E402
import trivy_amd.secret as S  # noqa: E402
from tests.test_scan_ext import _scan_patterns  # noqa: E402

ANY = (1 << 64) - 1


def fold(b):
    return (b & 0x1F) | ((b >> 1) & 0x20)


def seqs_of(pats, k):
    out = []
    for lit, cols in pats.items():
        if any(ch >= 0x80 for ch in lit):  # fold-special sequences: k_fold_special's job
            continue
        s = ([1 << fold(c) for c in lit] + cols)[:8]
        out.append((s[:k] + [ANY] * (k - len(s))) if k else s)
    return out


def group_rate(flag):
    g = flag[: (len(flag) // 8) * 8].reshape(-1, 8).any(axis=1)
    return g.mean()


def exact(seqs, colt, k):
    n = len(colt) - 8
    fl = np.zeros(n, bool)
    for s in seqs:
        m = np.ones(n, bool)
        for j in range(k):
            m &= ((np.uint64(s[j]) >> colt[j:n + j].astype(np.uint64)) & np.uint64(1)).astype(bool)
        fl |= m
    return fl


def teddy(seqs, colt, k, nb, train):
    n = len(colt) - 8
    cA, cB = colt & 7, colt >> 3

    def tables(bucket):
        tA = np.zeros((k, 8), bool)
        tB = np.zeros((k, 8), bool)
        for s in bucket:
            for j in range(k):
                for c in range(64):
                    if (s[j] >> c) & 1:
                        tA[j, c & 7] = True
                        tB[j, c >> 3] = True
        return tA, tB

    def flags(bucket, lim):
        tA, tB = tables(bucket)
        m = np.ones(lim, bool)
        for j in range(k):
            m &= tA[j][cA[j:lim + j]] & tB[j][cB[j:lim + j]]
        return m

    single = [flags([s], train).mean() for s in seqs]
    buckets = [[] for _ in range(nb)]
    cur = [np.zeros(train, bool) for _ in range(nb)]
    for i in np.argsort(single)[::-1]:
        best = None
        for b in range(nb):
            f = flags(buckets[b] + [seqs[i]], train)
            cost = int(f.sum()) - int(cur[b].sum())
            if best is None or cost < best[0]:
                best = (cost, b, f)
        buckets[best[1]].append(seqs[i])
        cur[best[1]] = best[2]
    fl = np.zeros(n, bool)
    for bk in buckets:
        if bk:
            fl |= flags(bk, n)
    return fl


def stride2_bitmap(seqs_full, colt):
    bm = np.zeros(1 << 18, bool)

    def cols(m):
        return np.array([c for c in range(64) if (m >> c) & 1], dtype=np.int64)

    def add(a, b, c):
        A, Bc, C = cols(a), cols(b), cols(c)
        bm[(A[:, None, None] | (Bc[None, :, None] << 6) | (C[None, None, :] << 12)).ravel()] = True

    for s in seqs_full:
        if len(s) >= 4:
            add(s[0], s[1], s[2])
            add(s[1], s[2], s[3])
        elif len(s) == 3:
            add(s[0], s[1], s[2])
            add(s[1], s[2], ANY)
        elif len(s) == 2:
            add(s[0], s[1], ANY)
            add(ANY, s[0], s[1])
        else:
            add(s[0], ANY, ANY)
            add(ANY, s[0], ANY)
    n = len(colt) - 16
    q = np.arange(0, n, 2)
    key = colt[q] | (colt[q + 1] << 6) | (colt[q + 2] << 12)
    f = bm[key]
    flag = np.zeros(n, bool)
    flag[q[f]] = True
    # bank cost of the lookups: 32 lanes, each its own 4 KiB span (positions/2 per lane)
    lanes = 64 * 32
    m = len(q) // lanes * lanes
    dw = ((key >> 5) ^ ((key >> 12) & 31))[:m].reshape(lanes, -1)[:, :256]
    g = np.sort(dw.reshape(lanes // 32, 32, -1).transpose(0, 2, 1).reshape(-1, 32), axis=1)
    dist = np.ones_like(g, bool)
    dist[:, 1:] = g[:, 1:] != g[:, :-1]
    kk = np.where(dist, g % 32, 32)
    cnt = np.zeros((g.shape[0], 33), np.int32)
    np.add.at(cnt, (np.repeat(np.arange(g.shape[0]), 32), kk.ravel()), 1)
    return flag, bm.mean(), cnt[:, :32].max(1).mean()


def main():
    regions = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    sc = S.new_scanner(None)
    pats, _, _ = _scan_patterns(sc._rs.handle)
    text = B.corpus(regions, 20261017)
    colt = fold(text.astype(np.int64))
    print(f"corpus {len(text)} bytes (bench text model), {len(pats)} scan patterns")
    for k in (2, 3, 4):
        print(f"exact {k}-prefix filter: flagged 8-byte groups {group_rate(exact(seqs_of(pats, k), colt, k)):.4f}")
    train = min(len(colt) - 8, 1 << 20)
    for nb, k in ((8, 3), (8, 4), (16, 4)):
        fl = teddy(seqs_of(pats, k), colt, k, nb, train)
        print(f"teddy {nb} buckets, {k} offsets: flagged 8-byte groups {group_rate(fl):.4f}")
    fl, fill, cyc = stride2_bitmap(seqs_of(pats, 0), colt)
    print(f"stride-2 3-gram bitmap: fill {fill:.4f}, flagged 8-byte groups {group_rate(fl):.4f}, "
          f"LDS cycles per 32-lane lookup {cyc:.2f} (x 0.5 lookups per byte)")
    print("k_scan_fast today: 1 lookup per byte at 2.96 cycles per 32-lane group (tools/bank_sim.py)")


if __name__ == "__main__":
    main()
