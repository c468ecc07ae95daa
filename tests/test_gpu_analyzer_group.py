"""The tagged build's secret analyzer (secret_mi355x.go, mirrored by
trivy_amd.analyzer.GPUSecretAnalyzer) inside Trivy's AnalyzerGroup on the
MI355X: real page-locked staging, tsg_analyze_staged batches, no oracle on
the product path (the oracle only computes the reference's expected secrets:
SecretAnalyzer.Analyze of every required file, secret.go:79-153).

* requirements.txt / sub/requirements.txt (claimed by a language analyzer)
  and usr/bin/tool.sh (an OS package's installed file) are secret-scanned as
  the reference's per-file analyzer scans them, while another post-analyzer's
  FS is filtered (analyzer.go:475-488);
* batches that span two artifacts analyzed at once keep each artifact's
  secrets its own;
* a failed GPU batch is re-scanned file by file on the GPU (one file per
  call): the artifact still gets every secret;
* a file larger than the staging, and a file that cannot be read after an
  earlier batch left a secret at its slot's offset."""
import io
import os
import threading

import pytest

from . import analyzer_tree as T

pytestmark = pytest.mark.gpu

S = pytest.importorskip("trivy_amd.secret")
N = pytest.importorskip("trivy_amd._native")
from trivy_amd import analyzer as A  # noqa: E402


def _registry(batch_bytes):
    reg = A.Registry()
    reg.register_analyzer(T.PipAnalyzer())
    reg.register_analyzer(T.DpkgAnalyzer())
    rec = T.RecordingPostAnalyzer()
    reg.register_post_analyzer("jar", rec.init)
    a = A.register_gpu_secret(reg, batch_bytes)  # no go_analyze: the GPU serves every path
    return reg, a, rec


def test_claimed_files_scanned_on_gpu(tmp_path):
    T.make_tree(str(tmp_path), 31, n=300)
    big = tmp_path / "big" / "huge.env"
    big.parent.mkdir()
    big.write_bytes(b"x = 1\n" * 40000 + f"token: {T.GHP}\n".encode())
    reg, a, rec = _registry(128 << 10)
    g = A.AnalyzerGroup.new(reg, A.AnalyzerOptions())
    res = A.inspect_local(str(tmp_path), g)
    want = T.reference_secrets(str(tmp_path))
    assert T.canon(res.secrets) == T.canon(want)
    paths = {s.FilePath for s in res.secrets}
    assert {"requirements.txt", "sub/requirements.txt", "usr/bin/tool.sh", "win/crlf.env", "big/huge.env"} <= paths
    assert "requirements.txt" not in rec.seen and "usr/bin/tool.sh" not in rec.seen
    assert a._gpu_err is None and len(want) > 50
    assert not a._results


def test_concurrent_artifacts_on_gpu(tmp_path):
    roots = [str(tmp_path / "a"), str(tmp_path / "b")]
    for k, r in enumerate(roots):
        os.makedirs(r)
        T.make_tree(r, 40 + k, n=150)
    reg, a, _ = _registry(48 << 10)
    groups = [A.AnalyzerGroup.new(reg, A.AnalyzerOptions()) for _ in roots]
    out = [None, None]

    def run(k):
        out[k] = A.inspect_local(roots[k], groups[k], parallel=4)
    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for k, r in enumerate(roots):
        assert T.canon(out[k].secrets) == T.canon(T.reference_secrets(r)), r
    assert not a._results


def test_failed_gpu_batch_rescanned_per_file(tmp_path, monkeypatch):
    T.make_tree(str(tmp_path), 33, n=150)
    reg, a, _ = _registry(64 << 10)
    g = A.AnalyzerGroup.new(reg, A.AnalyzerOptions())
    a._backend()
    batch = a._st.batch
    real = batch.analyze
    fails = {"n": 2}

    def flaky():
        if fails["n"]:
            fails["n"] -= 1
            raise N.EngineError(N.TSG_ERR_DEVICE, "injected batch failure")
        return real()
    monkeypatch.setattr(batch, "analyze", flaky)
    res = A.inspect_local(str(tmp_path), g)
    assert fails["n"] == 0
    assert T.canon(res.secrets) == T.canon(T.reference_secrets(str(tmp_path)))


def test_unreadable_file_after_a_batch_on_gpu():
    a = A.GPUSecretAnalyzer(batch_bytes=1 << 16)
    a.init(A.AnalyzerOptions())
    post = a.post_analyzer_init(A.AnalyzerOptions())
    body = f"x = 1\ntoken: {T.GHP}\n".encode()
    ia = A.FsFileInfo("a.env", len(body))
    assert post.required("a.env", ia)
    a.analyze_input(A.AnalysisInput("root", "a.env", ia, io.BytesIO(body)))
    got = post.post_analyze(A.MapFS())
    assert [s.FilePath for s in got.secrets] == ["a.env"] and len(got.secrets[0].Findings) == 1

    class Broken(io.BytesIO):
        def readinto(self, b):
            raise OSError("input/output error")
    ib = A.FsFileInfo("b.env", len(body))
    assert post.required("b.env", ib)
    with pytest.raises(OSError):
        a.analyze_input(A.AnalysisInput("root", "b.env", ib, Broken(b"y" * len(body))))
    assert post.post_analyze(A.MapFS()) is None
