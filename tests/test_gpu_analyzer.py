"""GPU parity of the batched SecretAnalyzer front end (tsg_analyze): the
utils.IsBinary gate (pkg/fanal/utils/utils.go:77-95), '\\r' deletion
(pkg/fanal/analyzer/secret/secret.go:91) and the '/' prefix (:95-98) ahead of
Scan, against the oracle's SecretAnalyzer.Analyze on raw files: CRLF text,
'\\r' inside secrets (they only match once stripped), CR-only files, control
bytes inside and past the 300-byte IsBinary head, empty and tiny files."""
import dataclasses
import random

import pytest

from oracle import secret_oracle as o

from . import corpus_gen

pytestmark = pytest.mark.gpu

S = pytest.importorskip("trivy_amd.secret")
from trivy_amd.analyzer import SecretAnalyzer  # noqa: E402


def _plain(res):
    if res is None:
        return None
    return [{"FilePath": s.FilePath, "Findings": sorted(
        (f.RuleID, f.StartLine, f.EndLine, f.Match, tuple((ln.Number, ln.Content) for ln in f.Code.Lines))
        for f in s.Findings)} for s in res]


def _oracle_plain(res):
    if res is None:
        return None
    return [{"FilePath": r["FilePath"], "Findings": sorted(
        (f.RuleID, f.StartLine, f.EndLine, f.Match, tuple((ln["Number"], ln["Content"]) for ln in f.Code["Lines"]))
        for f in r["Findings"])} for r in res]


def _raw_files(seed, n):
    rng = random.Random(seed)
    files = []
    for i, (p, d) in enumerate(corpus_gen.make_corpus(seed, n)):
        kind = i % 6
        if kind == 0:  # CRLF everywhere
            d = d.replace(b"\n", b"\r\n")
        elif kind == 1:  # stray CRs, some inside secrets
            b = bytearray(d)
            for _ in range(rng.randint(1, 20)):
                b.insert(rng.randrange(len(b) + 1), 0x0D)
            d = bytes(b)
        elif kind == 2:  # control byte in the IsBinary head -> skipped
            at = rng.randrange(min(len(d), 300)) if d else 0
            d = d[:at] + bytes([rng.choice([0, 1, 6, 11, 14, 26, 28, 31, 0x7F])]) + d[at:]
        elif kind == 3:  # control byte after the head -> scanned
            d = b"x" * 300 + b"\x01" + d
        files.append((p, d, rng.choice(["", "/src"])))
    files += [
        ("empty.txt", b"", ""),
        ("crs.txt", b"\r\r\r\r", ""),
        ("split.sh", b"export GH=ghp_" + b"\r".join(bytes([c]) for c in b"A1b2C3d4E5f6G7h8I9j0K1l2M3n4O5p6Q7r8") + b"\r\n", ""),
        ("esc.txt", b"\x1b[0m token ghp_" + b"Z" * 36 + b"\n", ""),  # ESC (27) is not a binary byte
        ("tab.txt", b"\t\x0b ghp_" + b"Y" * 36, ""),  # \v (11) is
        ("big_crlf.txt", b"".join(corpus_gen.make_file(rng, n_lines=200) for _ in range(20)).replace(b"\n", b"\r\n"), "d"),
    ]
    return files


@pytest.mark.parametrize("seed", [31, 32])
def test_analyze_batch_vs_oracle(seed):
    files = _raw_files(seed, 400)
    a = SecretAnalyzer()
    a.init("")
    got = a.analyze_batch(files)
    oa = o.SecretAnalyzer("")
    n_bin = n_found = 0
    for (p, d, dir_), g in zip(files, got):
        want = oa.analyze(p, d, dir_)
        n_bin += o.is_binary(d, len(d))
        n_found += want is not None
        assert _plain(g) == _oracle_plain(want), f"analyze mismatch on {p} (dir={dir_!r})"
    assert n_bin > 10 and n_found > 50


def test_analyze_no_cr_no_binary_fast_path():
    # nothing to strip: the batch is scanned in place (no compaction)
    files = [(p, d.replace(b"\r", b""), "") for p, d in corpus_gen.make_corpus(33, 200)]
    files = [(p, d, x) for p, d, x in files if not o.is_binary(d, len(d))]
    a = SecretAnalyzer()
    a.init("")
    got = a.analyze_batch(files)
    oa = o.SecretAnalyzer("")
    for (p, d, dir_), g in zip(files, got):
        assert _plain(g) == _oracle_plain(oa.analyze(p, d, dir_)), p
