"""Layer-tar walker (walker.LayerTar.Walk, pkg/fanal/walker/tar.go:35-117):
the native tsg_layer_tar_walk against the reference's own TestLayerTar_Walk
cases (tar_test.go:17-92 over testdata/test.tar, copied to
tests/golden/walker/test.tar) and against the oracle restatement (stdlib
tarfile reader) on generated GNU / PAX / USTAR layers with long names,
whiteouts, opaque dirs, links and skip globs.  CPU only: no compute call."""
import io
import os
import random
import tarfile

import pytest

from oracle import layertar_oracle as lo

W = pytest.importorskip("trivy_amd.walker")

GOLDEN_TAR = os.path.join(os.path.dirname(__file__), "golden", "walker", "test.tar")


def _native(layer, skip_files=(), skip_dirs=()):
    got = []
    opq, wh = W.LayerTar(skip_files, skip_dirs).walk(
        layer, lambda p, info, opener: got.append((p, info.size, info.is_dir, opener())))
    return got, opq, wh


def _oracle(layer, skip_files=(), skip_dirs=()):
    got = []
    opq, wh = lo.walk(layer, lambda p, size, is_dir, content: got.append((p, size, is_dir, content)),
                      skip_files, skip_dirs)
    return got, opq, wh


# --- reference known answers (tar_test.go:17-92) -----------------------------

@pytest.mark.parametrize("walker", ["native", "oracle"])
@pytest.mark.parametrize("case", [
    dict(name="happy path", opt={}),
    dict(name="skip file", opt=dict(skip_files=["/app/myweb/index.html"]), banned=lambda p: p == "app/myweb/index.html"),
    dict(name="skip dir", opt=dict(skip_dirs=["/app"]), banned=lambda p: p.startswith("app")),
])
def test_reference_layer_tar_walk(walker, case):
    data = open(GOLDEN_TAR, "rb").read()
    fn = _native if walker == "native" else _oracle
    got, opq, wh = fn(data, **case["opt"])
    assert opq == ["etc/"]
    assert wh == ["foo/foo"]
    banned = case.get("banned")
    if banned:
        assert not any(banned(p) for p, *_ in got)
    assert ("baz", 4, False, b"baz\n") in got


def test_reference_sad_path():
    def boom(*_):
        raise RuntimeError("error")
    with pytest.raises(W.WalkError, match="failed to analyze file"):
        W.LayerTar().walk(GOLDEN_TAR, boom)
    with pytest.raises(lo.WalkError, match="failed to analyze file"):
        lo.walk(open(GOLDEN_TAR, "rb").read(), boom)


def test_walk_from_path_and_buffer_agree():
    data = open(GOLDEN_TAR, "rb").read()
    assert _native(GOLDEN_TAR) == _native(data) == _native(bytearray(data)) == _oracle(data)


# --- generated layers vs the oracle --------------------------------------------

def _rand_name(rng, depth):
    comps = []
    for _ in range(depth):
        k = rng.random()
        if k < 0.05:
            comps.append("x" * rng.randint(60, 140))  # long component -> GNU 'L' / PAX path / USTAR prefix
        elif k < 0.1:
            comps.append(rng.choice([".git", "node_modules", "proc", "vendor", "etc", "app"]))
        else:
            comps.append("".join(rng.choice("abcdefgh_.-") for _ in range(rng.randint(1, 12))).strip(".") or "d")
    return "/".join(comps)


def make_layer(seed, n=120, fmt=tarfile.GNU_FORMAT):
    rng = random.Random(seed)
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w", format=fmt) as tf:
        for i in range(n):
            name = _rand_name(rng, rng.randint(1, 5))
            if fmt == tarfile.USTAR_FORMAT and (len(name) > 250 or any(len(c) > 99 for c in name.split("/"))):
                name = "/".join(c[:40] for c in name.split("/"))[:90]
            k = rng.random()
            lead = rng.choice(["", "", "./", "/"])
            if k < 0.08:
                ti = tarfile.TarInfo(lead + os.path.dirname(name) + "/.wh..wh..opq" if "/" in name else ".wh..wh..opq")
                tf.addfile(ti, io.BytesIO(b""))
            elif k < 0.16:
                d, b = os.path.split(name)
                ti = tarfile.TarInfo(lead + (d + "/" if d else "") + ".wh." + b)
                tf.addfile(ti, io.BytesIO(b""))
            elif k < 0.3:
                ti = tarfile.TarInfo(lead + name)
                ti.type = tarfile.DIRTYPE
                tf.addfile(ti)
            elif k < 0.36:
                ti = tarfile.TarInfo(lead + name)
                ti.type = rng.choice([tarfile.SYMTYPE, tarfile.LNKTYPE])
                ti.linkname = "y" * rng.randint(1, 90 if fmt == tarfile.USTAR_FORMAT else 150)
                tf.addfile(ti)
            else:
                body = bytes(rng.randrange(256) for _ in range(rng.choice([0, 1, 511, 512, 513, rng.randint(0, 4000)])))
                ti = tarfile.TarInfo(lead + name)
                ti.size = len(body)
                ti.mode = rng.choice([0o644, 0o755, 0o600])
                tf.addfile(ti, io.BytesIO(body))
    return buf.getvalue()


SKIPS = [
    dict(),
    dict(skip_dirs=["**/.git", "proc", "sys", "dev"]),
    dict(skip_dirs=["/app", "**/node_modules"], skip_files=["**/*.c", "etc/*"]),
    dict(skip_files=["**/{a,b}*", "[a-c]?_*"], skip_dirs=["vendor/**"]),
]


@pytest.mark.parametrize("fmt", [tarfile.GNU_FORMAT, tarfile.PAX_FORMAT, tarfile.USTAR_FORMAT])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_generated_layers_match_oracle(fmt, seed):
    data = make_layer(seed * 10 + fmt, fmt=fmt)
    for opt in SKIPS:
        assert _native(data, **opt) == _oracle(data, **opt), opt


def test_empty_layer():
    assert _native(b"") == ([], [], [])
    end = b"\0" * 1024
    assert _native(end) == _oracle(end) == ([], [], [])


def test_malformed_layers_fail_loudly():
    data = make_layer(7, n=10)
    with pytest.raises(W.WalkError, match="failed to extract the archive"):
        _native(data[:700])  # cut inside a member's data
    bad = bytearray(data)
    bad[0] ^= 0x41  # name byte changes -> checksum mismatch
    with pytest.raises(W.WalkError, match="failed to extract the archive"):
        _native(bytes(bad))


def test_zero_block_rules():
    """archive/tar readHeader: one zero block then EOF ends the walk, two zero
    blocks end it, a zero block followed by a header is ErrHeader ("invalid
    tar header"), a zero block followed by a partial block is unexpected EOF."""
    one = make_layer(8, n=3)
    body = one.rstrip(b"\0")
    body += b"\0" * ((-len(body)) % 512)
    z = b"\0" * 512
    assert _native(body + z)[0] == _native(one)[0]
    assert _native(body + z + z)[0] == _native(one)[0]
    with pytest.raises(W.WalkError, match="invalid tar header"):
        _native(body + z + make_layer(9, n=2))
    with pytest.raises(W.WalkError, match="unexpected EOF"):
        _native(body + z + b"x" * 100)


def test_fuzzed_layers_never_crash():
    """Random truncations and byte flips of generated layers: the walk either
    succeeds or reports "failed to extract the archive" (never aborts)."""
    rng = random.Random(99)
    ok = bad = 0
    for k in range(300):
        data = bytearray(make_layer(100 + k % 7, n=6, fmt=rng.choice([tarfile.GNU_FORMAT, tarfile.PAX_FORMAT])))
        for _ in range(rng.randint(1, 6)):
            data[rng.randrange(len(data))] = rng.randrange(256)
        if rng.random() < 0.3:
            data = data[: rng.randrange(len(data) + 1)]
        try:
            _native(bytes(data))
            ok += 1
        except W.WalkError as e:
            assert "failed to extract the archive" in str(e)
            bad += 1
    assert ok and bad


# --- doublestar.Match (walk.go:43) --------------------------------------------

GLOBS = [
    ("**/.git", [".git", "a/.git", "a/b/.git", "a/.gitx", "x.git"]),
    ("proc", ["proc", "proc/1", "xproc"]),
    ("a/**", ["a", "a/b", "a/b/c", "ab", "b/a"]),
    ("**", ["", "a", "a/b"]),
    ("**/*.go", ["x.go", "a/x.go", "a/b/x.go", "a/b/x.gox"]),
    ("*.go", ["x.go", "a/x.go"]),
    ("a/**/b", ["a/b", "a/x/b", "a/x/y/b", "a/xb", "ab"]),
    ("{a,b}/c", ["a/c", "b/c", "c/c", "ab/c"]),
    ("x{1,2{3,4}}", ["x1", "x23", "x24", "x2"]),
    ("[a-c]x", ["ax", "bx", "dx", "/x"]),
    ("[!a-c]x", ["ax", "dx", "/x"]),
    ("[^a]?", ["ba", "ab", "b/"]),
    ("\\*", ["*", "a"]),
    ("a?c", ["abc", "a/c", "ac"]),
    ("app/myweb/index.html", ["app/myweb/index.html", "app/myweb/index.htm"]),
]


@pytest.mark.parametrize("pattern,paths", GLOBS)
def test_glob_match_native_vs_oracle(pattern, paths):
    for p in paths:
        assert W.glob_match(pattern, p) == lo.doublestar_match(pattern, p), (pattern, p)


def test_bad_glob_pattern():
    with pytest.raises(Exception):
        W.glob_match("[abc", "a")
    with pytest.raises(ValueError):
        lo.doublestar_match("[abc", "a")


def test_allow_path_native_vs_oracle():
    from oracle import secret_oracle as o
    import trivy_amd.secret as S

    sc, osc = S.new_scanner(), o.Scanner(None)
    for p in ["usr/share/doc/x", "/usr/share/doc/x", "a/node_modules/b", "README.md", "app/test/x.go", "vendor/a",
              "src/vendor/a", "x/examples/y", "locale/fr.json", "usr/lib/python3/a.py", "src/main.go", ".md", "a/b"]:
        assert sc.allow_path(p) == osc.allow_path(p), p
