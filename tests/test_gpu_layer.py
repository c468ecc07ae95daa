"""GPU parity of one container-image layer through the batched analyzer
(trivy_amd.walker.analyze_layer): the native layer walk (walker/tar.go:35-117),
AnalyzeFile's directory skip + SecretAnalyzer.Required (analyzer.go:396-411,
secret.go:115-153) and ONE tsg_analyze call over spans of the layer buffer,
against the oracle's tarfile-based walk followed by per-file
SecretAnalyzer.Analyze with Dir "" (image.go:269), sorted by FilePath
(AnalysisResult.Sort, analyzer.go:218-229)."""
import io
import os
import random
import tarfile

import pytest

from oracle import layertar_oracle as lo
from oracle import secret_oracle as o

from . import corpus_gen
from .test_gpu_analyzer import _oracle_plain, _plain

pytestmark = pytest.mark.gpu

W = pytest.importorskip("trivy_amd.walker")
from trivy_amd.analyzer import SecretAnalyzer  # noqa: E402


def _layer(seed, n):
    rng = random.Random(seed)
    buf = io.BytesIO()
    dirs = ["app", "app/src", "etc", "usr/share/doc/pkg", "node_modules/x", ".git", "proc", "root/.ssh",
            "opt/" + "l" * 120]
    with tarfile.open(fileobj=buf, mode="w", format=rng.choice([tarfile.GNU_FORMAT, tarfile.PAX_FORMAT])) as tf:
        for d in dirs:
            ti = tarfile.TarInfo(d)
            ti.type = tarfile.DIRTYPE
            tf.addfile(ti)
        for i, (p, d) in enumerate(corpus_gen.make_corpus(seed, n)):
            k = i % 9
            if k == 0:
                d = d.replace(b"\n", b"\r\n")
            elif k == 1 and d:
                d = d[:50] + b"\x00" + d[50:]  # binary head -> skipped
            name = rng.choice(dirs) + "/" + p.replace("/", "_")
            if k == 2:
                name = rng.choice(dirs) + "/" + rng.choice(["go.sum", "yarn.lock", "logo.png", "a.pyc"])
            if k == 3:
                ti = tarfile.TarInfo(name + ".lnk")
                ti.type = tarfile.SYMTYPE
                ti.linkname = name
                tf.addfile(ti)
            ti = tarfile.TarInfo(name)
            ti.size = len(d)
            tf.addfile(ti, io.BytesIO(d))
        wh = tarfile.TarInfo("etc/.wh.passwd")
        tf.addfile(wh, io.BytesIO(b""))
    return buf.getvalue()


def _oracle_layer(data, skip_files=(), skip_dirs=(), config=""):
    oa = o.SecretAnalyzer(config)
    out = []

    def fn(path, size, is_dir, content):
        if is_dir or not oa.required(path, size):
            return
        res = oa.analyze(path, content, "")
        if res is not None:
            out.extend(res)
    opq, wh = lo.walk(data, fn, skip_files, skip_dirs)
    # AnalysisResult.Sort (analyzer.go:218-229): by FilePath, findings by (RuleID, StartLine)
    out.sort(key=lambda r: r["FilePath"])
    for r in out:
        r["Findings"].sort(key=lambda f: (f.RuleID, f.StartLine))
    return out, opq, wh


@pytest.mark.parametrize("seed,skip_dirs", [(41, ()), (42, tuple(W.DEFAULT_SKIP_DIRS)), (43, ("app/**",))])
def test_analyze_layer_vs_oracle(seed, skip_dirs, tmp_path):
    data = _layer(seed, 300)
    a = SecretAnalyzer()
    a.init("")
    want, wopq, wwh = _oracle_layer(data, skip_dirs=skip_dirs)
    got, opq, wh = W.analyze_layer(a, data, skip_dirs=skip_dirs)
    assert (opq, wh) == (wopq, wwh) == ([], ["etc/passwd"])
    assert _plain(got) == _oracle_plain(want)
    assert len(want) > 20
    # the same layer from a file (mmap'd, zero-copy spans)
    f = tmp_path / "layer.tar"
    f.write_bytes(data)
    got2, _, _ = W.analyze_layer(a, str(f), skip_dirs=skip_dirs)
    assert _plain(got2) == _plain(got)


def test_analyze_layer_reference_tar():
    a = SecretAnalyzer()
    a.init("")
    got, opq, wh = W.analyze_layer(a, os.path.join(os.path.dirname(__file__), "golden", "walker", "test.tar"))
    assert (got, opq, wh) == ([], ["etc/"], ["foo/foo"])


def test_analyze_layers_pipelined_matches_single():
    a = SecretAnalyzer()
    a.init("")
    layers = [_layer(50 + k, 120) for k in range(5)]
    got = W.analyze_layers(a, layers, skip_dirs=["proc"], walk_threads=3)
    assert len(got) == 5
    for data, (secs, opq, wh) in zip(layers, got):
        one, opq1, wh1 = W.analyze_layer(a, data, skip_dirs=["proc"])
        assert _plain(secs) == _plain(one) and (opq, wh) == (opq1, wh1)
        want, _, _ = _oracle_layer(data, skip_dirs=["proc"])
        assert _plain(secs) == _oracle_plain(want)


def test_analyze_layers_error_leaves_other_layers_intact():
    """A layer whose walk fails (a corrupt header) among layers that are being
    analyzed on both engines: the error surfaces as the walk error, every
    other walk is closed by its own analysis or, if never picked up, by the
    caller (no freed walk reaches tsg_analyze_layer), and the engines serve
    the next call with results equal to the oracle's."""
    a = SecretAnalyzer()
    a.init("")
    good = [_layer(60 + k, 150) for k in range(6)]
    bad = bytearray(good[1])
    bad[148:156] = b"99999999"  # header checksum no longer matches
    layers = [good[0], bytes(bad)] + good[2:]
    with pytest.raises(W.WalkError):
        W.analyze_layers(a, layers, walk_threads=3)
    got = W.analyze_layers(a, good[:3], walk_threads=3)
    for data, (secs, _, _) in zip(good[:3], got):
        want, _, _ = _oracle_layer(data)
        assert _plain(secs) == _oracle_plain(want)


def test_analyze_layers_base_layer_yields_no_secrets():
    """image.go:209-213: a base layer (its DiffID in the base image's) carries
    TypeSecret in its disabled list, so the reference's AnalyzeFile never calls
    the secret analyzer on its files.  The layer hook honours the same list:
    the base layer is walked (whiteouts and opaque dirs still count) and
    yields no secrets; the other layers are untouched."""
    a = SecretAnalyzer()
    a.init("")
    layers = [_layer(70 + k, 150) for k in range(3)]
    got = W.analyze_layers(a, layers, walk_threads=2, disabled=[True, False, True])
    for k, (data, (secs, opq, wh)) in enumerate(zip(layers, got)):
        want, wopq, wwh = _oracle_layer(data)
        assert (opq, wh) == (wopq, wwh)
        if k in (0, 2):
            assert secs == [] and len(want) > 5  # the layer had secrets; a base layer reports none
        else:
            assert _plain(secs) == _oracle_plain(want)


def test_analyze_layers_dead_extra_engine_falls_back_in_order(monkeypatch):
    """an extra engine failing with a device error hands its layer
    -- and every later layer queued on it -- to the first engine's queue; the
    results stay in input order and equal the oracle's, and every walk is
    closed (the next call works on both engines)."""
    import trivy_amd._native as N
    import trivy_amd.secret as S

    a = SecretAnalyzer()
    a.init("")
    engs = S.get_engines(a.scanner.device, 2)
    real = W._analyze_walked
    calls = {"dead": 0}

    def flaky(analyzer, addr, n, w, engine=None):
        if engine is not None and engine.value == engs[1].value:
            calls["dead"] += 1
            raise N.EngineError(N.TSG_ERR_DEVICE, "injected device error")
        return real(analyzer, addr, n, w, engine)

    monkeypatch.setattr(W, "_analyze_walked", flaky)
    layers = [_layer(80 + k, 100) for k in range(6)]
    got = W.analyze_layers(a, layers, walk_threads=3, engines=2)
    assert calls["dead"] == 1  # the engine is tried once, then skipped
    for data, (secs, _, _) in zip(layers, got):
        want, _, _ = _oracle_layer(data)
        assert _plain(secs) == _oracle_plain(want)
    monkeypatch.setattr(W, "_analyze_walked", real)
    again = W.analyze_layers(a, layers[:2], walk_threads=2, engines=2)
    assert [_plain(s) for s, _, _ in again] == [_plain(s) for s, _, _ in got[:2]]


def test_analyze_layer_finding_order():
    """Two findings of one rule whose Match order (Scan's sort) is the reverse
    of their line order: the layer result carries AnalysisResult.Sort's
    (RuleID, StartLine) order, compared as lists (no re-sorting here)."""
    content = b"x = 1\ntoken: ghp_" + b"Z" * 36 + b"\ny = 2\nauth: ghp_" + b"A" * 36 + b"\n"  # Match: "auth" < "token"
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w", format=tarfile.GNU_FORMAT) as tf:
        ti = tarfile.TarInfo("app/config.env")
        ti.size = len(content)
        tf.addfile(ti, io.BytesIO(content))
    data = buf.getvalue()
    a = SecretAnalyzer()
    a.init("")
    got, _, _ = W.analyze_layer(a, data)
    assert [(f.RuleID, f.StartLine) for f in got[0].Findings] == [("github-pat", 2), ("github-pat", 4)]
    want, _, _ = _oracle_layer(data)
    assert _plain(got) == _oracle_plain(want)


def test_analyze_layer_custom_rules_vs_oracle(tmp_path):
    """configs[3]'s workload names builtin + custom trivy-secret.yaml rules: a
    layer of stress-rule files (custom-rule instances, a minified line,
    binary-ish files) analysed with a 60-rule custom config, against the
    oracle's walk + Analyze with the same config."""
    from . import stress_rules

    rules = stress_rules.make_rules(777, 60)
    cfg = str(tmp_path / "trivy-secret.yaml")
    stress_rules.write_config(cfg, rules)
    files = stress_rules.make_corpus(778, rules, 120, long_line_bytes=40_000)
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w", format=tarfile.PAX_FORMAT) as tf:
        for p, d in files:
            ti = tarfile.TarInfo("app/" + p)
            ti.size = len(d)
            tf.addfile(ti, io.BytesIO(d))
    data = buf.getvalue()
    a = SecretAnalyzer()
    a.init(cfg)
    got, _, _ = W.analyze_layer(a, data)
    want, _, _ = _oracle_layer(data, config=cfg)
    assert _plain(got) == _oracle_plain(want)
    assert sum(f.RuleID.startswith("stress-") for s in got for f in s.Findings) > 50
