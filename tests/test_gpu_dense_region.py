"""Findings of dense files (at most 384 bytes per kept location: stored whole
in the arena's dense region, censored by k_dense_fill from the sorted
locations, engine.hip dense_begin / dense_issue) next to sparse files (their
lines as distinct-line segments), field by field against the oracle
(toFinding / findLocation / censorLocation, pkg/fanal/secret/scanner.go:454-537).

Many tiny files put several file groups inside one 256-byte fill step of a
lane (the group advance of k_dense_fill) and regions of 1..15 bytes of
padding; overlapping locations of two rules, a location ending on the file's
last byte, a file without a trailing newline, empty files and 16-byte
aligned sizes are all in the batch."""
import random

import pytest

from oracle import secret_oracle as o

from .test_gpu_parity import _canon, _oracle_plain, _plain

pytestmark = pytest.mark.gpu

S = pytest.importorskip("trivy_amd.secret")

CONFIG = r"""rules:
  - id: tok-long
    category: general
    title: tok long
    severity: HIGH
    regex: tok_[a-z0-9]{12}
    keywords:
      - tok_
  - id: tok-short
    category: general
    title: tok short
    severity: LOW
    regex: '_[a-z0-9]{6}x'
    keywords:
      - tok_
"""


def _tok(rng):
    return ("tok_" + "".join(rng.choice("abc0123456789") for _ in range(6)) + "x"
            + "".join(rng.choice("abc0123") for _ in range(5))).encode()


def _tiny(rng, i):
    kind = i % 7
    if kind == 0:
        return b""
    if kind == 1:  # the secret is the whole file, no newline
        return _tok(rng)
    if kind == 2:  # ends on the secret's last byte after a newline
        return b"a = 1\nv = " + _tok(rng)
    if kind == 3:  # padded to a 16-byte multiple
        body = b"x " + _tok(rng) + b"\n"
        return body + b"#" * ((-len(body)) % 16)
    if kind == 4:  # several on one line, overlapping rules
        return b" ".join(_tok(rng) for _ in range(rng.randint(2, 4))) + b"\n"
    if kind == 5:  # lines around the secret (Code lines 2 before / 1 after)
        return b"l1\nl2\nl3\nk = " + _tok(rng) + b"\nl5\nl6\n"
    return b"\n".join(b"n%d = " % j + _tok(rng) for j in range(rng.randint(1, 6)))


def _sparse(rng, kb):
    lines = [b"filler line %d with no secret at all" % j for j in range(kb * 25)]
    lines[rng.randrange(len(lines))] = b"k = " + _tok(rng)
    return b"\n".join(lines) + b"\n"


def test_gpu_dense_and_sparse_files_vs_oracle(tmp_path):
    cfg_path = str(tmp_path / "trivy-secret.yaml")
    with open(cfg_path, "w") as f:
        f.write(CONFIG)
    rng = random.Random(20261018)
    files = []
    for i in range(600):
        if i % 50 == 25:
            files.append((f"sparse/{i}.txt", _sparse(rng, rng.randint(2, 8))))
        else:
            files.append((f"tiny/{i}.txt", _tiny(rng, i)))
    sc = S.new_scanner(S.parse_config(cfg_path))
    got = sc.scan_batch_device([S.ScanArgs(p, d) for p, d in files])
    oracle = o.Scanner(o.parse_config(cfg_path))
    n_find = 0
    for (p, d), g in zip(files, got):
        want = _oracle_plain(oracle.scan(p, d))
        n_find += len(want["Findings"])
        assert _canon(_plain(g)) == _canon(want), p
    assert n_find > 1000
