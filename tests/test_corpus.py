"""The synthetic corpus generator (bench_gen/corpus.hip, host twin) against
the oracle: every builtin rule has a template, every real plant is found by
Scanner.Scan at its recorded location, no decoy (one char short, EXAMPLE
allow-listed) is, and the 0.1 % non-ASCII files carry K/ſ/İ/é runes.  This is
what lets bench.py check planted == found on the full-size corpus."""
import collections
import ctypes

import numpy as np
import pytest

from oracle import secret_oracle as O

N = pytest.importorskip("trivy_amd._native")

PLANT = np.dtype([("file", "<u4"), ("tpl", "<u4"), ("start", "<u8"), ("end", "<u8"), ("decoy", "<u4"),
                  ("pad", "<u4")])


def _gen(seed, f, n, dens):
    buf = (ctypes.c_uint8 * max(1, n))()
    pl = np.zeros(4096, dtype=PLANT)
    npl = ctypes.c_size_t()
    N.check(N.gen.tsg_gen_file_plants(seed, f, n, dens, buf, pl.ctypes.data, len(pl), ctypes.byref(npl)))
    return bytes(buf)[:n], pl[:min(npl.value, len(pl))]


def _rules():
    return [N.gen.tsg_gen_template_rule(i).decode() for i in range(N.gen.tsg_gen_template_count())]


def test_one_template_per_builtin_rule():
    assert N.gen.tsg_gen_plant_record_size() == PLANT.itemsize
    assert sorted(_rules()) == sorted(r.id for r in O.Scanner(None).rules)


def test_plants_match_oracle():
    rules = _rules()
    sc = O.Scanner(None)
    seen, miss, decoys = collections.Counter(), [], 0
    for f in range(260):
        data, pl = _gen(123, f, 20000 + (f * 7919) % 60000, 3e-4)
        got = {(x.RuleID, x.Start, x.End) for x in sc.scan("src/a.go", data, with_offsets=True)["Findings"]}
        for p in pl:
            key = (rules[p["tpl"]], int(p["start"]), int(p["end"]))
            if p["decoy"] == 0:
                seen[key[0]] += 1
                if key not in got:
                    miss.append(key)
            elif p["decoy"] in (1, 2):
                decoys += 1
                assert key not in got and (key[0], key[1], key[2] - 1) not in got, f"decoy found: {key}"
    assert not miss, miss[:5]
    assert len(seen) == len(rules), set(rules) - set(seen)
    assert decoys > 100


def test_nonascii_files():
    seed = 20261017
    files = [f for f in range(20000) if N.gen.tsg_gen_file_nonascii(seed, f)]
    assert 5 <= len(files) <= 45  # 0.1 %
    hi = special = 0
    for f in files:
        data, pl = _gen(seed, f, 30000, 1e-6)
        hi += max(data) >= 0x80
        special += any(s in data for s in ("K".encode(), "ſ".encode(), "İ".encode()))
    assert hi >= len(files) * 0.7 and special >= len(files) // 2
    # K/ſ-spelled rule instances appear (their expectation is the oracle's, not the generator's)
    kinds = collections.Counter()
    for f in files[:200]:
        for k in range(4):
            _, pl = _gen(seed, f, 4_000_000 if k == 0 else 200_000 + k, 1e-6)
            kinds.update(int(x) for x in pl["decoy"])
    assert kinds[3] > 0
