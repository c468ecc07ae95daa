"""The tagged build's secret analyzer inside Trivy's AnalyzerGroup, on the CPU
(trivy_amd.analyzer mirrors analyzer.go and secret_mi355x.go; the GPU variant
of these checks is tests/test_gpu_analyzer_group.py):

* files other analyzers claim (an Application's FilePath, SystemInstalledFiles)
  are still secret-scanned, while every post-analyzer's FS is filtered as in
  analyzer.go:475-488;
* post-analyzer initialisers run before the disabled check
  (analyzer.go:358-365) and the disabled secret analyzer never creates an
  engine nor parses its config;
* no usable GPU: Trivy's per-file Scan, identical results;
* the staging/flush/identity logic with a host stand-in for the page-locked
  staging (a bytearray reused across batches, as the real one is): batches
  that span files of two concurrent artifacts, a failed batch re-scanned per
  file, a file that cannot be read (its slot is zeroed: no stale secret of
  an earlier batch under its path), a file larger than the staging."""
import io
import os
import threading

import pytest

import trivy_amd._native as N
import trivy_amd.secret as S
from trivy_amd import analyzer as A

from . import analyzer_tree as T


def _registry(go_analyze, batch_bytes=64 << 10):
    reg = A.Registry()
    reg.register_analyzer(T.PipAnalyzer())
    reg.register_analyzer(T.DpkgAnalyzer())
    rec = T.RecordingPostAnalyzer()
    reg.register_post_analyzer("jar", rec.init)
    a = A.register_gpu_secret(reg, batch_bytes, go_analyze)
    return reg, a, rec


class HostStaging:
    """Stand-in for S.Batch (tsg_staging_*) on the CPU: contiguous slots in
    one bytearray that every batch reuses from offset 0, analyzed by Trivy's
    per-file Analyze (the oracle)."""

    def __init__(self, capacity, go_analyze):
        self.cap, self.go = capacity, go_analyze
        self.buf = bytearray(capacity)
        self.used, self.paths, self.slots = 0, [], []
        self.fail_next = 0
        self.runs = 0

    def __len__(self):
        return len(self.paths)

    def reserve(self, path, size):
        if self.used + size + 1 > self.cap:
            return None
        mv = memoryview(self.buf)[self.used:self.used + size]
        self.used += size + 1
        self.paths.append(path)
        self.slots.append(mv)
        return mv

    def analyze(self):
        self.runs += 1
        if self.fail_next:
            self.fail_next -= 1
            raise N.EngineError(N.TSG_ERR_DEVICE, "injected batch failure")
        out = []
        for p, mv in zip(self.paths, self.slots):
            r = self.go(p, bytes(mv), "dir")  # (paths already carry the Dir == "" prefix)
            out.append(r[0] if r else None)
        self.reset()
        return out

    def reset(self):
        self.used, self.paths, self.slots = 0, [], []

    def close(self):
        pass


@pytest.fixture
def no_gpu(monkeypatch):
    def fail(*a, **k):
        raise N.EngineError(N.TSG_ERR_NO_DEVICE, "no device (test)")
    monkeypatch.setattr(S, "get_engine", fail)


@pytest.fixture
def host_staging(monkeypatch):
    made = []
    go = T.oracle_go_analyze()

    def new_batch(self, capacity):
        b = HostStaging(capacity, go)
        made.append(b)
        return b
    monkeypatch.setattr(S.Scanner, "new_batch", new_batch)
    # a file larger than the staging goes alone through tsg_analyze: the same
    # per-file Analyze here
    monkeypatch.setattr(S.Scanner, "analyze_batch",
                        lambda self, batch: [(lambda r: r[0] if r else None)(go(a.file_path, a.content, "dir"))
                                             for a in batch])
    return made


def test_claimed_files_are_scanned_without_gpu(tmp_path, no_gpu):
    T.make_tree(str(tmp_path), 7)
    reg, a, rec = _registry(T.oracle_go_analyze())
    g = A.AnalyzerGroup.new(reg, A.AnalyzerOptions())
    res = A.inspect_local(str(tmp_path), g)
    want = T.reference_secrets(str(tmp_path))
    assert T.canon(res.secrets) == T.canon(want)
    paths = {s.FilePath for s in res.secrets}
    assert {"requirements.txt", "sub/requirements.txt", "usr/bin/tool.sh", "win/crlf.env"} <= paths
    # the other post-analyzer's FS was filtered (analyzer.go:475-488)
    assert rec.seen is not None and "requirements.txt" not in rec.seen and "usr/bin/tool.sh" not in rec.seen
    assert "win/crlf.env" in rec.seen
    assert {x.type for x in res.applications} == {"pip"} and len(res.applications) == 2
    assert a._gpu_err is not None  # the per-file fallback served every file


def test_disabled_secret_creates_no_engine(tmp_path, monkeypatch):
    T.make_tree(str(tmp_path), 8, n=20)
    calls = []
    monkeypatch.setattr(N.lib, "tsg_engine_create", lambda *a: calls.append(a) or N.TSG_ERR_NO_DEVICE)
    def engine_requested(*a, **k):
        calls.append(a)
        raise AssertionError("engine requested")
    monkeypatch.setattr(S, "get_engine", engine_requested)
    reg, a, rec = _registry(T.oracle_go_analyze())
    inits = []
    real_init = reg.post_analyzers["secret"]
    reg.post_analyzers["secret"] = lambda opts: inits.append(opts) or real_init(opts)
    g = A.AnalyzerGroup.new(reg, A.AnalyzerOptions(disabled_analyzers=["secret"]))
    assert inits, "post-analyzer initialisers run before the disabled check (analyzer.go:358-365)"
    assert all(x.type() != "secret" for x in g.analyzers + g.post_analyzers)
    res = A.inspect_local(str(tmp_path), g)
    assert res.secrets == [] and calls == []
    assert a.scanner is None  # Init never ran: no config parsed, no ruleset compiled


def test_concurrent_artifacts_keep_their_own_secrets(tmp_path, host_staging):
    """Two filesystem artifacts analyzed at once by the one process-wide
    analyzer, a staging so small that every batch mixes their files: each
    artifact gets exactly its own secrets (FileInfo identity)."""
    roots = [str(tmp_path / "a"), str(tmp_path / "b")]
    for k, r in enumerate(roots):
        os.makedirs(r)
        T.make_tree(r, 20 + k, n=80)
    reg, a, _ = _registry(T.oracle_go_analyze(), batch_bytes=24 << 10)
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
    assert host_staging[0].runs > 4
    assert not a._results  # every result was handed to its walk


def test_failed_batch_is_rescanned_per_file(tmp_path, host_staging):
    T.make_tree(str(tmp_path), 9, n=80)
    reg, a, _ = _registry(T.oracle_go_analyze(), batch_bytes=32 << 10)
    g = A.AnalyzerGroup.new(reg, A.AnalyzerOptions())
    a.init(A.AnalyzerOptions())
    a._backend()
    host_staging[0].fail_next = 2
    res = A.inspect_local(str(tmp_path), g)
    assert T.canon(res.secrets) == T.canon(T.reference_secrets(str(tmp_path)))
    assert host_staging[0].fail_next == 0


def test_unreadable_file_leaves_no_stale_bytes(host_staging):
    """A file that cannot be read into its slot after an earlier batch put a
    secret at the same staging offset: the slot is zeroed (IsBinary skips
    it), the read error surfaces (AnalyzeFile logs and drops it), and the
    file reports nothing -- not the earlier file's secret."""
    a = A.GPUSecretAnalyzer(batch_bytes=4096, go_analyze=T.oracle_go_analyze())
    a.init(A.AnalyzerOptions())
    post = a.post_analyzer_init(A.AnalyzerOptions())
    body = f"x = 1\ntoken: {T.GHP}\n".encode()
    ia = A.FsFileInfo("a.env", len(body))
    assert post.required("a.env", ia)
    a.analyze_input(A.AnalysisInput("root", "a.env", ia, io.BytesIO(body)))
    got = post.post_analyze(A.MapFS())
    assert [s.FilePath for s in got.secrets] == ["a.env"]

    class Broken(io.BytesIO):
        def readinto(self, b):
            raise OSError("input/output error")
    ib = A.FsFileInfo("b.env", len(body))
    assert post.required("b.env", ib)
    with pytest.raises(OSError):
        a.analyze_input(A.AnalysisInput("root", "b.env", ib, Broken(b"y" * len(body))))
    assert post.post_analyze(A.MapFS()) is None


def test_file_larger_than_staging_and_file_patterns(tmp_path, host_staging):
    """A file larger than the whole staging goes alone; a file linked only
    through --file-patterns (Required never asked, analyzer.go:457) is picked
    up from the post-analyzer's FS by file identity."""
    T.make_tree(str(tmp_path), 11, n=30)
    big = tmp_path / "big" / "huge.env"
    big.parent.mkdir()
    big.write_bytes(b"x = 1\n" * 20000 + f"token: {T.GHP}\n".encode())
    # a skipped extension a file pattern brings back in
    (tmp_path / "keys.pyc").write_bytes(f"# {T.GHP}\n".encode())
    reg, a, _ = _registry(T.oracle_go_analyze(), batch_bytes=32 << 10)
    g = A.AnalyzerGroup.new(reg, A.AnalyzerOptions(file_patterns=["secret:\\.pyc$"]))
    res = A.inspect_local(str(tmp_path), g)
    got = {s.FilePath: s for s in res.secrets}
    assert "big/huge.env" in got and "keys.pyc" in got
    oa = T.oracle_go_analyze()
    want_pyc = oa("keys.pyc", (tmp_path / "keys.pyc").read_bytes(), str(tmp_path))
    assert T.canon([got["keys.pyc"]]) == T.canon(want_pyc)
    assert not a._results
