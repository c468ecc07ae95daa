"""Caller-filled staging (tsg_staging_*, tsg_analyze_staged / tsg_scan_staged)
and the tagged Go build's post-analyzer that drives it
(integration/go/pkg/fanal/analyzer/secret/secret_mi355x.go, mirrored by
trivy_amd.analyzer.SecretPostAnalyzer): files read straight into page-locked
memory give the same findings as the packing entry points and as the oracle's
per-file Analyze (pkg/fanal/analyzer/secret/secret.go:79-113)."""
import os

import pytest

from oracle import secret_oracle as o

from . import corpus_gen
from .test_gpu_parity import _canon, _oracle_plain, _plain

pytestmark = pytest.mark.gpu

S = pytest.importorskip("trivy_amd.secret")
N = pytest.importorskip("trivy_amd._native")
from trivy_amd.analyzer import SecretAnalyzer, SecretPostAnalyzer  # noqa: E402


def _files(seed, n):
    files = corpus_gen.make_corpus(seed, n)
    for i in range(0, len(files), 7):  # CRLF and binary heads, as Analyze sees raw files
        p, d = files[i]
        files[i] = (p, d.replace(b"\n", b"\r\n"))
    files.append(("bin/tool.dat", b"\x00\x01ghp_" + b"a" * 36))
    return files


def _fill(data):
    def f(dst):
        dst[:] = data
    return f


def test_staged_analyze_and_scan_equal_packing_entry_points():
    sc = S.new_scanner(None)
    files = _files(31, 300)
    args = [S.ScanArgs(p, d) for p, d in files]
    want_a = sc.analyze_batch(args)
    stripped = [S.ScanArgs(p, d.replace(b"\r", b"")) for p, d in files]
    want_s = sc.scan_batch(stripped)
    with sc.new_batch(64 << 20) as b:
        for p, d in files:
            assert b.add(p, len(d), _fill(d))
        got_a = b.analyze()
        assert len(b) == 0  # reset after the run
        for a in stripped:
            assert b.add(a.file_path, len(a.content), _fill(a.content))
        got_s = b.scan()
    assert [None if g is None else _plain(g) for g in got_a] == [None if w is None else _plain(w) for w in want_a]
    assert [_plain(g) for g in got_s] == [_plain(w) for w in want_s]
    assert sum(len(w.Findings) for w in want_s) > 100


def test_staging_full_and_refill():
    """TSG_ERR_FULL when a file does not fit; the batch runs, resets and the
    file goes in on the next round; a file larger than the whole buffer
    never fits."""
    sc = S.new_scanner(None)
    files = _files(32, 120)
    cap = 64 << 10
    got, pending = [], []
    with sc.new_batch(cap) as b:
        for p, d in files:
            if len(d) + 1 > cap:
                assert not b.add(p, len(d), _fill(d))
                continue
            if not b.add(p, len(d), _fill(d)):
                got += [(q, r) for q, r in zip(pending, b.analyze())]
                pending = []
                assert b.add(p, len(d), _fill(d))
            pending.append(p)
        got += [(q, r) for q, r in zip(pending, b.analyze())]
    want = {p: w for (p, _), w in zip(files, sc.analyze_batch([S.ScanArgs(p, d) for p, d in files]))}
    assert len(got) > 60
    for p, g in got:
        assert (None if g is None else _plain(g)) == (None if want[p] is None else _plain(want[p])), p


def test_post_analyzer_equals_per_file_analyze(tmp_path):
    """PostAnalyze over the post-analyzer FS -- the files Required accepted,
    linked by the artifact walk (artifact/local/fs.go:100-106) -- with a small
    staging (several batches, one file larger than the staging alone) == the
    oracle's per-file Analyze with Dir set (no '/' prefix), in walk order."""
    from trivy_amd.analyzer import _walk_dir

    files = _files(33, 200)
    files.append(("big/huge.env", b"x = 1\n" * 30000 + b"token: ghp_" + b"Q" * 36 + b"\n"))
    a = SecretAnalyzer()
    a.init("")
    post = SecretPostAnalyzer(a, batch_bytes=128 << 10)
    n_req = 0
    for p, d in files:
        if not post.required(p, len(d)):
            continue
        n_req += 1
        f = tmp_path / p
        f.parent.mkdir(parents=True, exist_ok=True)
        f.write_bytes(d)
    got = post.post_analyze(str(tmp_path))
    oa = o.SecretAnalyzer("")
    want = []
    for p, _ in _walk_dir(str(tmp_path)):
        r = oa.analyze(p, open(os.path.join(tmp_path, p), "rb").read(), str(tmp_path))
        if r:
            want.extend(r)
    assert [_canon(_plain(g)) for g in got] == [_canon(_oracle_plain(w)) for w in want]
    assert any(g.FilePath == "big/huge.env" for g in got)
    assert n_req > 150 and len(want) > 50
