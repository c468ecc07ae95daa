#!/usr/bin/env python3
"""k_scan_big over the 64 fold columns instead of byte classes (CPU study):
the configs[4] scan patterns as an Aho-Corasick automaton over fold6
columns (k_scan_fast's ALU alphabet), its state count, the columns used,
and cold-state visits per byte on the bench text model for dense-row budgets
(128-byte rows).  Compare tools/big_visits.py (class alphabet, 92-byte rows)."""
import sys, ctypes, numpy as np, collections
sys.path.insert(0,'/root/repo/tools'); sys.path.insert(0,'/root/repo')
import bank_sim as B
import trivy_amd._native as N, trivy_amd.secret as S
from tests import stress_rules
from tests.test_scan_ext import _scan_patterns
srules = stress_rules.make_rules(20261019, 1000)
stress_rules.write_config("/tmp/stress.yaml", srules)
sc = S.new_scanner(S.parse_config("/tmp/stress.yaml"))
pats, _, _ = _scan_patterns(sc._rs.handle)
st=[ctypes.c_uint32() for _ in range(4)]; fp=ctypes.c_int()
N.check(N.lib.tsg_ruleset_stats(sc._rs.handle, *[ctypes.byref(x) for x in st], ctypes.byref(fp)))
print("class AC states", st[0].value, "classes", st[1].value, "patterns", len(pats))
depth = 8
fold = lambda b: (b & 0x1F) | ((b >> 1) & 0x20)
lits = [bytes(l[:depth]) for l in pats if all(c < 0x80 for c in l)]
print("ascii lits", len(lits), "non-ascii", len(pats) - len(lits))
# trie over columns
go = [dict()]; out = [False]
for l in lits:
    s = 0
    for c in l:
        v = fold(c)
        if v not in go[s]:
            go[s][v] = len(go); go.append(dict()); out.append(False)
        s = go[s][v]
    out[s] = True
S_ = len(go)
fail = [0]*S_; depth_of=[0]*S_
q = collections.deque()
delta = np.zeros((S_, 64), np.int32)
for v in range(64):
    t = go[0].get(v, 0); delta[0, v] = t
    if t: q.append(t); depth_of[t]=1
order=[0]
while q:
    s = q.popleft(); order.append(s)
    out[s] = out[s] or out[fail[s]]
    for v in range(64):
        t = go[s].get(v)
        if t is not None:
            fail[t] = delta[fail[s], v]; depth_of[t]=depth_of[s]+1; q.append(t); delta[s, v] = t
        else:
            delta[s, v] = delta[fail[s], v]
print("column AC states", S_)
used = sorted({fold(c) for l in lits for c in l})
print("used columns", len(used))
text = np.frombuffer(bytes(B.corpus(64, 20261017)), np.uint8)
cols = ((text & 0x1F) | ((text >> 1) & 0x20)).astype(np.int64)
vis = np.zeros(S_, np.int64)
s = 0
# walk (python loop over 8MB is slow; take 2MB)
n = 2_000_000
for i in range(n):
    s = delta[s, cols[i]]
    vis[s] += 1
# rank by bfs order (depth) as product does
rank = np.argsort(np.argsort([depth_of[x] for x in range(S_)], kind='stable'))
bydepth = np.array(order)
for nd in (900, 1000, 1100, 1200, 1400, 1600):
    dense = set(bydepth[:nd].tolist())
    cold = sum(vis[x] for x in range(S_) if x not in dense)
    print(f"dense rows {nd} ({nd*128/1024:.0f} KB): cold visits per byte {cold/n:.5f}")
# diff-edge counts for cold states
ne = [sum(1 for v in range(64) if delta[x,v]!=delta[fail[x],v]) for x in range(S_)]
print("states with >2 edges:", sum(1 for x in ne if x>2), "list words", sum(x+1 for x in ne if x>2))
