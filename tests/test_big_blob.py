"""k_scan_big's LDS blob (engine.hip BigDev: dense rows of the likeliest
states, 8-byte cold-state records, overflow lists) replayed on the CPU
against the keyword/anchor automaton's own table, for the 1000-rule stress
set (configs[4]) under both state numberings: every step must reach the same
state with the same output bit, so the device walk (same code shape) equals
the table walk of k_scan_generic."""
import ctypes
import random

import pytest

from . import stress_rules

S = pytest.importorskip("trivy_amd.secret")
N = pytest.importorskip("trivy_amd._native")


@pytest.fixture(scope="module")
def stress_rs(tmp_path_factory):
    rules = stress_rules.make_rules(20261019, 1000)
    path = str(tmp_path_factory.mktemp("stress") / "trivy-secret.yaml")
    stress_rules.write_config(path, rules)
    files = stress_rules.make_corpus(7, rules, 30, long_line_bytes=20_000)
    return S.new_scanner(S.parse_config(path)), files


def _check(sc, text, bfs):
    mm, hops, nd = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32()
    N.check(N.lib.tsg_ruleset_big_check(sc._rs.handle, text, len(text), bfs, ctypes.byref(mm), ctypes.byref(hops),
                                        ctypes.byref(nd)))
    return mm.value, hops.value, nd.value


@pytest.mark.parametrize("bfs", [0, 1])
def test_big_blob_walk_equals_table(stress_rs, bfs):
    sc, files = stress_rs
    rng = random.Random(5)
    text = b"".join(d for _, d in files)
    text += bytes(rng.randrange(256) for _ in range(200_000))  # every class, non-ASCII too
    text += bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz_-=: \n0123456789") for _ in range(200_000))
    mm, hops, nd = _check(sc, text, bfs)
    assert nd > 0
    assert mm == 0, f"{mm} steps disagree (bfs={bfs})"
    assert hops > 0  # the cold records are exercised


def test_big_blob_builtin_automaton():
    """The builtin automaton in the same blob shape (k_scan_fast's image is
    what scans it; the blob layout must still hold for any automaton)."""
    sc = S.new_scanner(None)
    rng = random.Random(9)
    text = bytes(rng.randrange(256) for _ in range(100_000)) + b"AKIA ghp_ sk_live_ -----BEGIN xoxb- " * 200
    for bfs in (0, 1):
        mm, hops, nd = _check(sc, text, bfs)
        assert nd > 0 and mm == 0


@pytest.mark.parametrize("kind", [1, 2, 3, 4])
def test_forged_blob_is_rejected(stress_rs, kind):
    """A malformed blob is an error, never a device walk that cannot end: the
    validator the engine runs before every upload (and tsg_ruleset_compile
    before handing out a ruleset) rejects a cold record whose ancestor row is
    not a dense row (kind 1), an unterminated overflow list and out-of-range
    entries / classes, and accepts the ruleset's real blob."""
    sc, _ = stress_rs
    rc = ctypes.c_int(-1)
    N.check(N.lib.tsg_ruleset_big_forge_check(sc._rs.handle, 0, ctypes.byref(rc)))
    assert rc.value == N.TSG_OK
    rc = ctypes.c_int(-1)
    N.check(N.lib.tsg_ruleset_big_forge_check(sc._rs.handle, kind, ctypes.byref(rc)))
    assert rc.value == N.TSG_ERR_INTERNAL


@pytest.mark.parametrize("floor", [0, 512])
def test_global_cold_records_blob(tmp_path, floor):
    """With a low LDS floor for the cold records the blob takes more dense
    rows and leaves the deep states' records to global memory
    (BigLds::gcold): the replay still equals the table, and the validator
    accepts the blob and rejects its forgeries."""
    prev = ctypes.c_uint32()
    N.check(N.lib.tsg_big_cold_lds_floor(floor, ctypes.byref(prev)))
    try:
        rules = stress_rules.make_rules(20261019, 1000)
        path = str(tmp_path / "trivy-secret.yaml")
        stress_rules.write_config(path, rules)
        sc = S.new_scanner(S.parse_config(path))
        files = stress_rules.make_corpus(11, rules, 20, long_line_bytes=10_000)
        rng = random.Random(6)
        text = b"".join(d for _, d in files) + bytes(rng.randrange(256) for _ in range(100_000))
        mm, hops, nd = _check(sc, text, 0)
        assert mm == 0 and hops > 0
        for kind in (0, 1, 2, 3, 4):
            rc = ctypes.c_int(-1)
            N.check(N.lib.tsg_ruleset_big_forge_check(sc._rs.handle, kind, ctypes.byref(rc)))
            assert rc.value == (N.TSG_OK if kind == 0 else N.TSG_ERR_INTERNAL)
    finally:
        N.check(N.lib.tsg_big_cold_lds_floor(prev.value, None))
    assert prev.value == 4096
    _, _, nd_default = _check(S.new_scanner(S.parse_config(path)), text[:1000], 0)
    assert nd > nd_default  # the low floor bought dense rows
