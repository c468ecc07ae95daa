"""Container-image layer walker: the mirror of walker.LayerTar
(pkg/fanal/walker/tar.go:23-117, walk.go:28-53) over the native
tsg_layer_tar_walk, plus `analyze_layer`, which hands every required regular
file of a layer to the GPU analyzer in ONE tsg_analyze call (SURVEY.md §8f
rank 2: batch submission instead of one Scan per file from --parallel
goroutines).

The layer is a host buffer (bytes, bytearray, mmap) or a path, which is
mmap'd read-only; file contents are spans of it, never copied here.
"""
from __future__ import annotations

import ctypes
import mmap
import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _native as N
from .types import Secret

Layer = Union[bytes, bytearray, memoryview, mmap.mmap, str, os.PathLike]

# walker.defaultSkipDirs (walk.go:17-22) — applied by the fs/image artifacts,
# not by LayerTar itself; exported for callers that want Trivy's defaults.
DEFAULT_SKIP_DIRS = ["**/.git", "proc", "sys", "dev"]


class WalkError(RuntimeError):
    pass


@dataclass(frozen=True)
class FileInfo:
    """The fs.FileInfo fields the analyzers read (hdr.FileInfo(), tar.go:85)."""
    name: str
    size: int
    mode: int
    is_dir: bool


def glob_match(pattern: str, path: str) -> bool:
    """doublestar.Match (walk.go:43), natively.  Raises on a bad pattern."""
    m = ctypes.c_int()
    N.check(N.lib.tsg_glob_match(pattern.encode(), path.encode(), ctypes.byref(m)))
    return bool(m.value)


def _open_layer(layer: Layer):
    """(buffer, base address, length, closer) for a layer without copying it."""
    if isinstance(layer, (str, os.PathLike)):
        f = open(layer, "rb")
        size = os.fstat(f.fileno()).st_size
        if size == 0:
            f.close()
            return b"", 0, 0, lambda: None
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)

        def close():
            mm.close()
            f.close()
        buf = mm
    else:
        buf, close = layer, (lambda: None)
    n = len(memoryview(buf).cast("B")) if not isinstance(buf, (bytes, bytearray, mmap.mmap)) else len(buf)
    addr = int(np.frombuffer(buf, dtype=np.uint8).ctypes.data) if n else 0
    return buf, addr, n, close


def _cstrs(v: Sequence[str]):
    arr = (ctypes.c_char_p * max(1, len(v)))(*[s.encode("utf-8", "surrogateescape") for s in v])
    return arr, len(v)


class _Walk:
    """Native walk (tsg_layer_tar_walk).  Entry tuples (path, offset, size,
    mode, is_dir) are materialised on first use only: the batched analyze
    needs none of them, just the paths of files that carry findings."""

    def __init__(self, addr: int, n: int, skip_files: Sequence[str], skip_dirs: Sequence[str]):
        sf, nsf = _cstrs(skip_files)
        sd, nsd = _cstrs(skip_dirs)
        self.handle = ctypes.c_void_p()
        rc = N.lib.tsg_layer_tar_walk(addr or None, n, sf, nsf, sd, nsd, ctypes.byref(self.handle))
        if rc != 0:
            raise WalkError(N.lib.tsg_last_error().decode("utf-8", "replace"))
        h = self.handle
        self.count = N.lib.tsg_tar_walk_entry_count(h)
        self._ents = N.lib.tsg_tar_walk_entries(h)
        self._entries = None
        self.opq_dirs = [N.lib.tsg_tar_walk_opq_dir(h, i).decode("utf-8", "surrogateescape")
                         for i in range(N.lib.tsg_tar_walk_opq_count(h))]
        self.wh_files = [N.lib.tsg_tar_walk_wh_file(h, i).decode("utf-8", "surrogateescape")
                         for i in range(N.lib.tsg_tar_walk_wh_count(h))]

    def path(self, i: int) -> str:
        e = self._ents[i]
        return ctypes.string_at(e.path, e.path_len).decode("utf-8", "surrogateescape")

    @property
    def entries(self) -> List[Tuple[str, int, int, int, bool]]:
        if self._entries is None:
            out = []
            for i in range(self.count):
                e = self._ents[i]
                out.append((self.path(i), e.offset, e.size, e.mode, bool(e.is_dir)))
            self._entries = out
        return self._entries

    def close(self):
        if self.handle:
            N.lib.tsg_tar_walk_free(self.handle)
            self.handle = ctypes.c_void_p()
            self._ents = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class _KeptBatch:
    """The analyze batch of one layer, lazily: item k is ScanArgs("/" + path
    of walk entry kept[k]), built only when a result needs its FilePath."""

    def __init__(self, walk: _Walk, kept, n: int):
        self.walk, self.kept, self.n = walk, kept, n

    def __len__(self):
        return self.n

    def __getitem__(self, k):
        from .secret import ScanArgs

        return ScanArgs("/" + self.walk.path(self.kept[k]), b"")


class LayerTar:
    """walker.LayerTar: NewLayerTar(Option{SkipFiles, SkipDirs}) (tar.go:28-33)."""

    def __init__(self, skip_files: Sequence[str] = (), skip_dirs: Sequence[str] = ()):
        self.skip_files = list(skip_files)
        self.skip_dirs = list(skip_dirs)

    def walk(self, layer: Layer,
             analyze_fn: Callable[[str, FileInfo, Callable[[], bytes]], None]) -> Tuple[List[str], List[str]]:
        """Walk (tar.go:35-90): analyze_fn(file_path, info, opener) for every
        directory and regular file that survives the skip rules, in archive
        order; returns (opqDirs, whFiles).  An analyze_fn error ends the walk
        with "failed to process the file: failed to analyze file: ..."."""
        buf, addr, n, close = _open_layer(layer)
        view = memoryview(buf).cast("B") if n else None
        try:
            with _Walk(addr, n, self.skip_files, self.skip_dirs) as w:
                w.entries  # noqa: B018 — materialise before the handle closes
            for path, off, size, mode, is_dir in w.entries:
                info = FileInfo(path.rsplit("/", 1)[-1], size, mode, is_dir)
                try:
                    analyze_fn(path, info, lambda o=off, s=size: bytes(view[o:o + s]))
                except Exception as e:  # noqa: BLE001 — mirrors the Go error wrap
                    raise WalkError(f"failed to process the file: failed to analyze file: {e}") from e
            return w.opq_dirs, w.wh_files
        finally:
            if n:
                view.release()
            del buf
            close()


def _analyze_walked(analyzer, addr: int, n: int, w: _Walk, engine=None) -> List[Secret]:
    from .secret import get_engine

    sc = analyzer.scanner
    if not w.handle:
        raise WalkError("layer walk already closed")
    kept = (ctypes.c_uint32 * max(1, w.count))()
    nk = ctypes.c_size_t()
    res = ctypes.c_void_p()
    eng = engine if engine is not None else get_engine(sc.device)
    N.check(N.lib.tsg_analyze_layer(eng, sc._rs.handle, addr or None, n, w.handle,
                                    (analyzer.config_path or "").encode(), kept, ctypes.byref(nk),
                                    ctypes.byref(res)))
    try:
        out = sc._convert(res, _KeptBatch(w, kept, nk.value))
    finally:
        N.lib.tsg_result_free(res)
    secrets = [r for r in out if r is not None and r.Findings]
    # AnalysisResult.Sort (analyzer.go:218-229): secrets by FilePath, then each
    # secret's findings by (RuleID, StartLine) -- Scan left them by (RuleID, Match)
    secrets.sort(key=lambda s: s.FilePath)
    for sec in secrets:
        sec.Findings.sort(key=lambda f: (f.RuleID, f.StartLine))
    return secrets


def analyze_layer(analyzer, layer: Layer, skip_files: Sequence[str] = (),
                  skip_dirs: Sequence[str] = ()) -> Tuple[List[Secret], List[str], List[str]]:
    """One image layer through the secret analyzer, batched: the layer walk
    (tar.go:35-90), then tsg_analyze_layer — AnalyzerGroup.AnalyzeFile's
    directory skip and SecretAnalyzer.Required (analyzer.go:396-411,
    secret.go:115-153) natively, and Analyze of every required file in one
    tsg_analyze call over spans of the layer buffer, with Dir == "" (the image
    artifact, image.go:269) so paths get the '/' prefix (secret.go:95-98).
    Returns (secrets sorted by FilePath as AnalysisResult.Sort does,
    analyzer.go:218-229, opqDirs, whFiles)."""
    return analyze_layers(analyzer, [layer], skip_files, skip_dirs, walk_threads=1)[0]


def analyze_layers(analyzer, layers: Sequence[Layer], skip_files: Sequence[str] = (),
                   skip_dirs: Sequence[str] = (), walk_threads: int = 4, engines: int = 2,
                   disabled: Sequence[bool] = ()) -> List[Tuple[List[Secret], List[str], List[str]]]:
    """The layers of an image (image.go:242-331 inspects them concurrently),
    pipelined: up to `walk_threads` native walks run ahead on host threads
    (ctypes drops the GIL), and layer k is analyzed on engine k % `engines`
    of the same GPU (secret.get_engines: own stream and buffers), each engine
    fed by its own single-worker queue, so one layer's host-to-device staging
    -- the PCIe-bound part -- overlaps the Required pass, scan pipeline and
    findings of the layer before it.  An extra engine holds its own device
    scratch and pinned staging: a layer whose analysis fails
    on an extra engine with a device error (e.g. out of memory) is re-run on
    the first engine -- on the first engine's own queue, so it never runs
    beside that queue's layers -- and that extra engine takes no more layers
    of this call (its queued layers go to the first queue too).
    `disabled[k]` true: secret scanning is disabled for layer k -- a base
    layer of the image (image.go:209-213 passes TypeSecret in the per-layer
    disabled list): the layer is walked (its opaque dirs and whiteouts are
    still needed) but not analyzed, and it yields no secrets.
    One (secrets, opqDirs, whFiles) per layer, in input order."""
    from concurrent.futures import ThreadPoolExecutor

    from .secret import get_engines

    engs = get_engines(analyzer.scanner.device, max(1, min(engines, len(layers))))
    opened = [_open_layer(x) for x in layers]
    dead = set()  # extra engines that failed with a device error

    def on(e, k, w):
        _, addr, n, _ = opened[k]
        return (_analyze_walked(analyzer, addr, n, w, engs[e]), w.opq_dirs, w.wh_files)

    def one(k, f):
        e = k % len(engs)
        with f.result() as w:  # this task owns the walk: closed here, whatever happens
            if k < len(disabled) and disabled[k]:
                return ([], w.opq_dirs, w.wh_files)
            if e != 0 and e not in dead:
                try:
                    return on(e, k, w)
                except N.EngineError as err:
                    if err.code != N.TSG_ERR_DEVICE:
                        raise
                    dead.add(e)
            if e == 0:
                return on(0, k, w)
            # a dead extra engine's layer: run on the first engine's queue (this
            # worker waits; the first queue never waits on another)
            return queues[0].submit(on, 0, k, w).result()

    pool = ThreadPoolExecutor(max_workers=max(1, walk_threads))
    queues = [ThreadPoolExecutor(max_workers=1) for _ in engs]
    futs, afuts = [], []
    try:
        futs = [pool.submit(_Walk, addr, n, skip_files, skip_dirs) for _, addr, n, _ in opened]
        afuts = [queues[k % len(engs)].submit(one, k, f) for k, f in enumerate(futs)]
        return [a.result() for a in afuts]
    finally:
        # on an error: analyses not started are cancelled, running ones are
        # waited for (each closes its own walk), and only walks that no
        # analysis picked up are freed here
        for a in afuts:
            a.cancel()
        for q in queues:
            q.shutdown(wait=True)
        pool.shutdown(wait=True)
        for k, f in enumerate(futs):
            if (k >= len(afuts) or afuts[k].cancelled()) and f.exception() is None:
                f.result().close()
        for buf, _, _, close in opened:
            del buf
            close()
