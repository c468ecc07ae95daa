"""k_scan_big with the deep cold-state records in global memory
(engine.hip BigLds::gcold): the cold-record LDS floor is set to 0
(tsg_big_cold_lds_floor), so the blob holds the most dense rows and nearly
every cold record is read from global memory; the 1000-rule stress set
(configs[4]'s automaton) is scanned and every file's findings are compared
with the oracle field by field."""
import ctypes

import pytest

from . import stress_rules

pytestmark = pytest.mark.gpu

S = pytest.importorskip("trivy_amd.secret")
N = pytest.importorskip("trivy_amd._native")


def test_big_global_cold_records_vs_oracle(tmp_path):
    from oracle import secret_oracle as o

    from .test_gpu_parity import _canon, _oracle_plain, _plain
    rules = stress_rules.make_rules(20261019, 1000)
    path = str(tmp_path / "trivy-secret.yaml")
    stress_rules.write_config(path, rules)
    files = stress_rules.make_corpus(91, rules, 24, long_line_bytes=20_000)
    prev = ctypes.c_uint32()
    N.check(N.lib.tsg_big_cold_lds_floor(0, ctypes.byref(prev)))
    try:
        sc = S.new_scanner(S.parse_config(path), device=0)
        got = sc.scan_batch([S.ScanArgs(p, d) for p, d in files])
    finally:
        N.check(N.lib.tsg_big_cold_lds_floor(prev.value, None))
    oracle = o.Scanner(o.parse_config(path))
    n = 0
    for (p, d), g in zip(files, got):
        want = _oracle_plain(oracle.scan(p, d))
        n += len(want["Findings"])
        assert _canon(_plain(g)) == _canon(want), p
    assert n > 100
