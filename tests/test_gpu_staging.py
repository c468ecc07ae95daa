"""Caller-filled staging (tsg_staging_*, tsg_analyze_staged / tsg_scan_staged):
files read straight into page-locked memory give the same findings as the
packing entry points.  The tagged Go build's analyzer that drives it inside
Trivy's AnalyzerGroup is tested in tests/test_gpu_analyzer_group.py."""
import pytest

from . import corpus_gen
from .test_gpu_parity import _plain

pytestmark = pytest.mark.gpu

S = pytest.importorskip("trivy_amd.secret")
N = pytest.importorskip("trivy_amd._native")


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


def test_reserve_failure_zeroes_slot():
    """Batch.add: a fill that raises leaves its slot zeroed -- the slot of a
    reset batch holds the previous batch's bytes until written -- so the
    file scans as binary instead of as an earlier file's content."""
    sc = S.new_scanner(None)
    body = b"x = 1\ntoken: ghp_" + b"K" * 36 + b"\n"
    with sc.new_batch(1 << 16) as b:
        assert b.add("a.env", len(body), _fill(body))
        first = b.analyze()
        assert first[0] is not None and len(first[0].Findings) == 1

        def broken(dst):  # writes nothing: the slot still holds a.env's bytes
            raise OSError("input/output error")
        with pytest.raises(OSError):
            b.add("b.env", len(body), broken)
        assert b.analyze() == [None]  # binary: NUL bytes
