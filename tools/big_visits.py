#!/usr/bin/env python3
"""k_scan_big dense-row study (CPU): cold-state visits per byte of the
configs[4] automaton (1000 stress rules + builtin) on the bench text model,
with the product blob (depth, then byte-model probability) and with a dense
set chosen by visit frequency on another seed of the same text (an upper
bound for any frequency-trained selection).  tsg_ruleset_ac_visits."""
import sys, ctypes, numpy as np
sys.path.insert(0,'/root/repo/tools'); sys.path.insert(0,'/root/repo')
import bank_sim as B
import trivy_amd._native as N, trivy_amd.secret as S
from tests import stress_rules

srules = stress_rules.make_rules(20261019, 1000)
stress_rules.write_config("/tmp/stress.yaml", srules)
sc = S.new_scanner(S.parse_config("/tmp/stress.yaml"))
st=[ctypes.c_uint32() for _ in range(4)]; fp=ctypes.c_int()
N.check(N.lib.tsg_ruleset_stats(sc._rs.handle, *[ctypes.byref(x) for x in st], ctypes.byref(fp)))
S_=st[0].value
train = bytes(B.corpus(64, 1234))
test = bytes(B.corpus(64, 20261017))
def visits(t):
    c=(ctypes.c_uint64*S_)(); nd=ctypes.c_uint32()
    N.check(N.lib.tsg_ruleset_ac_visits(sc._rs.handle, t, len(t), 1, c, S_, ctypes.byref(nd)))
    return np.frombuffer(c, np.uint64).astype(np.int64), nd.value
vt, nd = visits(train); vs, _ = visits(test)
n = len(test)
print("states", S_, "dense", nd, "bytes", n)
print("current blob: cold visits per byte", vs[nd:].sum()/n)
order = np.argsort(-vt)
dense_set = set(order[:nd].tolist()) | {0}
cold = sum(vs[i] for i in range(S_) if i not in dense_set)
print("train-frequency dense set: cold visits per byte", cold/n)
# how many distinct states visited at all
print("states visited in test:", (vs>0).sum(), " top-nd coverage of visits:", np.sort(vs)[::-1][:nd].sum()/vs.sum())

# cold visits per byte if the blob's dense region (its own order) held more rows
for nd2 in (1202, 1400, 1680, 2000, 2445):
    print(f"dense rows {nd2}: cold visits per byte {vs[nd2:].sum() / n:.5f}")
