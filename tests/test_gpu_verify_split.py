"""The verify split (k_verify_fast -> k_verify_slow -> k_allow, engine.hip)
on small batches.  The engine takes the split only for long job lists
(configs[4]-sized); tsg_engine_force_verify_split routes every list through
it, so the parity cases below -- builtin fuzz corpora, the golden configs
(allow rules, custom rules, exclude blocks), non-ASCII edge files (deferred
jobs), the empty-match fuzz rules and the 1000-rule stress set -- compare the
split's findings with the oracle field by field."""
import os
import random

import pytest

from . import corpus_gen, stress_rules
from .conftest import GOLDEN

pytestmark = pytest.mark.gpu

S = pytest.importorskip("trivy_amd.secret")
N = pytest.importorskip("trivy_amd._native")


@pytest.fixture(autouse=True)
def forced_split():
    eng = S.get_engine(0)
    N.check(N.lib.tsg_engine_force_verify_split(eng, 1))
    yield
    N.check(N.lib.tsg_engine_force_verify_split(eng, 0))


def test_split_builtin_fuzz_and_edges_vs_oracle():
    from .test_gpu_parity import _compare_batch
    rng = random.Random(23)
    files = corpus_gen.make_corpus(4242, 800)
    files += [("kelvin.txt", "token: ghp_K".encode() + b"A" * 35 + b"\nsk_live_" + b"a" * 20),
              ("longs.txt", "ſk_live_abcdefghijklmnop\nAWS_SECRET_KEY: ".encode() + b"B" * 40),
              ("idot.txt", "İİ key=\"".encode() + b"C" * 40 + b'"\n'),
              ("uni.txt", "é aws_secret_key = ".encode() + "Éa".encode() * 20 + b"\n"),
              ("invalid.txt", b"\xff\xfeghp_" + b"Z" * 36 + b"\xc3")]
    files += [(f"r{i}.txt", bytes(rng.randrange(256) for _ in range(rng.randint(0, 400)))) for i in range(40)]
    assert _compare_batch(files, seed_info="split") > 500


def test_split_golden_configs_vs_oracle():
    import json

    from .test_gpu_parity import _compare_batch
    cases = json.load(open(os.path.join(GOLDEN, "scanner_cases.json")))["cases"]
    for cfg in sorted({c["config"] for c in cases}):
        files = corpus_gen.make_corpus(hash(cfg) & 0xFFFF, 120)
        for c in cases:
            files.append((c["file_path"], open(os.path.join(GOLDEN, c["input"]), "rb").read().replace(b"\r", b"")))
        _compare_batch(files, os.path.join(GOLDEN, cfg), seed_info="split " + cfg)


def test_split_empty_match_rules_vs_oracle():
    from .test_gpu_empty_match import HAND, _hand_texts, _run, _selected
    from oracle import secret_oracle as o
    cases = _selected()[:60] + [(p, o.GoRegexp(p), _hand_texts()) for p in HAND]
    rules = [S.Rule(id=f"sp-{i:03d}", category="Fuzz", title="split", severity="HIGH", regex=pat,
                    path=r"^src/s%04d\.txt$" % i, keywords=[] if i % 3 else [next((c for c in pat if c.isalpha()), "a")])
             for i, (pat, _, _) in enumerate(cases)]
    files = [(f"src/s{i:04d}.txt", b"\n".join(c[2])) for i, c in enumerate(cases)]
    n, empty = _run(rules, files)
    assert n > 1000 and empty > 500


def test_split_stress_rules_vs_oracle(tmp_path):
    from oracle import secret_oracle as o

    from .test_gpu_parity import _canon, _oracle_plain, _plain
    rules = stress_rules.make_rules(20261019, 300)
    path = str(tmp_path / "trivy-secret.yaml")
    stress_rules.write_config(path, rules)
    files = stress_rules.make_corpus(77, rules, 40, long_line_bytes=30_000)
    sc = S.new_scanner(S.parse_config(path), device=0)
    got = sc.scan_batch([S.ScanArgs(p, d) for p, d in files])
    oracle = o.Scanner(o.parse_config(path))
    n = 0
    for (p, d), g in zip(files, got):
        want = _oracle_plain(oracle.scan(p, d))
        n += len(want["Findings"])
        assert _canon(_plain(g)) == _canon(want), p
    assert n > 100
