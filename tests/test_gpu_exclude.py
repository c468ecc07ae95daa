"""Exclude blocks on the device (Blocks.Match / find, pkg/fanal/secret/scanner.go:232-270,413-419):
a 10 k-file batch with global and per-rule exclude-block regexes -- (?s) spans,
line-anchored (?m) blocks, a block reached by several rules' locations, blocks
that contain a location only partly -- scanned through the C ABI and compared
field by field with the CPU oracle.  The containment filter runs on the device
(k_exclude_tags, k_excl_filter): no location leaves it before the findings."""
import os
import random

import pytest

from oracle import secret_oracle as o

from . import corpus_gen
from .test_gpu_parity import _canon, _oracle_plain, _plain

pytestmark = pytest.mark.gpu

S = pytest.importorskip("trivy_amd.secret")

CONFIG = r"""rules:
  - id: kv-secret
    category: general
    title: key value secret
    severity: HIGH
    regex: (?i)(?P<key>(secret|passwd))(=|:).{0,5}['"](?P<secret>[0-9a-zA-Z\-_=]{8,64})['"]
    secret-group-name: secret
    exclude-block:
      description: rule blocks
      regexes:
        - (?s)--- ignore kv start ---.*?--- ignore kv stop ---
        - '#\s*kv-ok[^\n]*\n[^\n]*'
  - id: tok-any
    category: general
    title: tok token
    severity: LOW
    regex: tok_[a-z0-9]{12}
    keywords:
      - tok_
exclude-block:
  description: global
  regexes:
    - --- ignore block start ---(.|\s)*?--- ignore block stop ---
    - (?m)^.*# nosecret$
"""


def _corpus(seed, n):
    rng = random.Random(seed)
    files = corpus_gen.make_corpus(seed, n)
    out = []
    for path, data in files:
        lines = data.split(b"\n")
        for _ in range(rng.randint(0, 3)):
            j = rng.randrange(len(lines) + 1)
            kind = rng.random()
            if kind < 0.3:
                v = "".join(rng.choice("abcdefghijk0123456789") for _ in range(rng.randint(6, 20)))
                lines.insert(j, (rng.choice(["secret", "PASSWD", "Secret"]) + rng.choice(["=", ":"]) + " '" + v
                                 + "'").encode())
            elif kind < 0.45:
                lines.insert(j, ("tok_" + "".join(rng.choice("abc0123456789") for _ in range(12))).encode())
            elif kind < 0.6:
                k = rng.randint(1, 4)
                lines[j:j + k] = [b"--- ignore block start ---"] + lines[j:j + k] + [b"--- ignore block stop ---"]
            elif kind < 0.75:
                k = rng.randint(1, 4)
                lines[j:j + k] = [b"--- ignore kv start ---"] + lines[j:j + k] + [b"--- ignore kv stop ---"]
            elif kind < 0.85 and lines:
                j = min(j, len(lines) - 1)
                lines[j] = lines[j] + b" # nosecret"
            else:
                lines.insert(j, b"# kv-ok reviewed")
        out.append((path, b"\n".join(lines)))
    return out


def test_gpu_exclude_blocks_10k_files_vs_oracle(tmp_path):
    cfg_path = str(tmp_path / "trivy-secret.yaml")
    with open(cfg_path, "w") as f:
        f.write(CONFIG)
    files = _corpus(20261017, 10000)
    sc = S.new_scanner(S.parse_config(cfg_path))
    got = sc.scan_batch([S.ScanArgs(p, d) for p, d in files])
    oracle = o.Scanner(o.parse_config(cfg_path))
    n_find = n_excl_files = 0
    bad = []
    for (p, d), g in zip(files, got):
        want = _oracle_plain(oracle.scan(p, d))
        n_find += len(want["Findings"])
        n_excl_files += b"ignore" in d or b"nosecret" in d or b"kv-ok" in d
        if _canon(_plain(g)) != _canon(want):
            bad.append(p)
    assert not bad, bad[:5]
    assert n_find > 1000 and n_excl_files > 1000
    # the blocks did remove findings: the same batch without them finds more
    plain_cfg = str(tmp_path / "no-blocks.yaml")
    with open(plain_cfg, "w") as f:
        f.write(CONFIG.split("exclude-block:\n  description: global")[0].replace(
            "    exclude-block:\n      description: rule blocks\n      regexes:\n"
            "        - (?s)--- ignore kv start ---.*?--- ignore kv stop ---\n"
            "        - '#\\s*kv-ok[^\\n]*\\n[^\\n]*'\n", ""))
    sc2 = S.new_scanner(S.parse_config(plain_cfg))
    got2 = sc2.scan_batch([S.ScanArgs(p, d) for p, d in files])
    assert sum(len(x.Findings) for x in got2) > sum(len(x.Findings) for x in got)
