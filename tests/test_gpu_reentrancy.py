"""Concurrent tsg_scan / tsg_analyze through the C ABI (the
ABI is thread-safe; a compiled ruleset is shared read-only, an engine
serialises the calls made on it).  Six host threads scan different batches at
once — three on one shared engine, three on private engines of the same GPU —
with one ruleset shared by all, and every result must equal the single-threaded
result of the same batch (findings field by field)."""
import ctypes
import threading

import pytest

from tests import corpus_gen

pytestmark = pytest.mark.gpu

N = pytest.importorskip("trivy_amd._native")
S = pytest.importorskip("trivy_amd.secret")


def _findings(sc, eng, fn, batch):
    files = (N.FileC * len(batch))()
    keep = []
    for i, (p, d) in enumerate(batch):
        buf = ctypes.create_string_buffer(d, len(d))
        keep.append(buf)
        files[i].data = ctypes.cast(buf, ctypes.c_void_p)
        files[i].len = len(d)
        files[i].path = p.encode()
    res = ctypes.c_void_p()
    N.check(fn(eng, sc._rs.handle, files, len(batch), ctypes.byref(res)))
    try:
        return sc._convert(res, [S.ScanArgs(p, d) for p, d in batch])
    finally:
        N.lib.tsg_result_free(res)


def test_concurrent_scans_equal_sequential():
    sc = S.new_scanner(None, device=0)
    shared = S.get_engine(0)
    private = []
    for _ in range(3):
        h = ctypes.c_void_p()
        N.check(N.lib.tsg_engine_create(0, ctypes.byref(h)))
        private.append(h)
    batches = [corpus_gen.make_corpus(9000 + k, 48) for k in range(6)]
    fns = [N.lib.tsg_scan, N.lib.tsg_analyze]
    want = [_findings(sc, shared, fns[k % 2], b) for k, b in enumerate(batches)]
    assert sum(len(s.Findings) for w in want for s in w) > 0
    got, errors = {}, []

    def worker(k):
        try:
            eng = shared if k < 3 else private[k - 3]
            for _ in range(3):
                r = _findings(sc, eng, fns[k % 2], batches[k])
                if r != want[k]:
                    errors.append(f"thread {k}: differs from the sequential result")
                    return
            got[k] = True
        except Exception as e:  # noqa: BLE001
            errors.append(f"thread {k}: {e!r}")

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    for h in private:
        N.lib.tsg_engine_free(h)
    assert not errors, errors
    assert len(got) == 6
