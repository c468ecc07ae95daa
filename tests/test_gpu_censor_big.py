"""Censoring of files with thousands of findings (censorLocation over every
kept location of a file, pkg/fanal/secret/scanner.go:425-462; line numbers on
the censored content, :481-503): files with >= 4096 locations are merged by
k_censor_big (a 1024-lane block per file) instead of one wave.  Overlapping
locations of two rules, secrets with newlines inside (private keys: their
censored newlines shift every later line number) and a minified line are
compared field by field with the oracle, next to small files in the same
batch (the wave path)."""
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

PEM = b"MIIEowIBAAKCAQEAu1SU1LfVLPHCozMxH2Mo4lgOEePzNm0tRgeLezV6ffAt0gunVTLw7onLRnrq0"


def _big_file(rng, n_lines, minified=False):
    parts = []
    for i in range(n_lines):
        x = rng.random()
        if x < 0.45:
            t = "".join(rng.choice("abc0123456789") for _ in range(6)) + "x" + \
                "".join(rng.choice("abc0123") for _ in range(5))
            parts.append(b"v = tok_" + t.encode())  # both rules: overlapping locations
        elif x < 0.7:
            parts.append(b"gh = ghp_" + bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyzABCDEF0123456789")
                                             for _ in range(36)))
        elif x < 0.72 and not minified:
            parts.append(b"-----BEGIN RSA PRIVATE KEY-----\n" + b"\n".join([PEM] * rng.randint(1, 4))
                         + b"\n-----END RSA PRIVATE KEY-----")
        else:
            parts.append(b"filler line %d with no secret" % i)
    return (b";" if minified else b"\n").join(parts) + b"\n"


def test_gpu_files_with_thousands_of_findings_vs_oracle(tmp_path):
    cfg_path = str(tmp_path / "trivy-secret.yaml")
    with open(cfg_path, "w") as f:
        f.write(CONFIG)
    rng = random.Random(99)
    files = [("small/a.txt", _big_file(rng, 40)),
             ("big/one.txt", _big_file(rng, 12000)),
             ("small/b.txt", _big_file(rng, 300)),
             ("big/two.txt", _big_file(rng, 9000)),
             ("min/app.min.js", _big_file(rng, 8000, minified=True)),
             ("small/c.txt", _big_file(rng, 5))]
    sc = S.new_scanner(S.parse_config(cfg_path))
    got = sc.scan_batch_device([S.ScanArgs(p, d) for p, d in files])
    oracle = o.Scanner(o.parse_config(cfg_path))
    sizes = []
    for (p, d), g in zip(files, got):
        want = _oracle_plain(oracle.scan(p, d))
        sizes.append(len(want["Findings"]))
        assert _canon(_plain(g)) == _canon(want), p
    assert max(sizes) >= 4096 * 2 and sum(s >= 4096 for s in sizes) >= 3, sizes
