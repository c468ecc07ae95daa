"""Mirror of the drop-in boundary: Trivy's SecretAnalyzer
(pkg/fanal/analyzer/secret/secret.go:28-153), utils.IsBinary
(pkg/fanal/utils/utils.go:77-95), the AnalyzerGroup that drives analyzers and
post-analyzers (pkg/fanal/analyzer/analyzer.go:93-107,315-370,396-503), the
filesystem artifact's walk (pkg/fanal/artifact/local/fs.go:70-125), and the
tagged Go build's GPU secret analyzer
(integration/go/pkg/fanal/analyzer/secret/secret_mi355x.go), mirrored line for
line by GPUSecretAnalyzer.

How the tagged build keeps Trivy's contract (analyzer.go):

* secrets stay a per-file ``analyzer``: AnalyzeFile calls Required and then
  Analyze for every file -- including files another analyzer claims
  (requirements.txt, pom.xml, ...), which AnalyzerGroup.PostAnalyze filters
  out of every post-analyzer's FS (analyzer.go:475-488) -- and honours the
  per-call ``disabled`` list (image base layers, image.go:209-213);
* Analyze does not scan: it reads the file straight into the process's
  page-locked GPU staging buffer (tsg_staging_add) and returns; a full buffer
  is analyzed on the GPU (tsg_analyze_staged) by the Analyze call that finds
  it full, and the results are kept per file, keyed by the file's
  os.FileInfo (the walker's value, which AnalyzeFile passes to both Analyze
  and RequiredPostAnalyzers);
* a post-analyzer of the same type exists only to learn when the walk is
  over: its Required records the walk's FileInfos (the same predicate as the
  analyzer's Required), and PostAnalyze -- called after wg.Wait()
  (fs.go:112-118) -- analyzes what is still staged and returns exactly the
  results of ITS files, so concurrent artifacts never see each other's
  secrets.  The filtered FS it is handed is only used to pick up files that
  reached it through --file-patterns (Required is skipped for those,
  analyzer.go:457);
* post-analyzer initialisers run before the disabled check
  (analyzer.go:358-365), so the initialiser creates nothing; the GPU engine
  is created at the first Analyze (never for ``--scanners vuln``), and a host
  without a usable GPU (no device, or a ruleset the engine returns
  TSG_ERR_UNSUPPORTED for) keeps Trivy's own per-file Scan;
* a GPU batch that fails is re-scanned file by file from the staged bytes
  (Trivy's Scan in the Go build), so one bad batch never aborts the artifact,
  as AnalyzeFile drops a failing file's error (analyzer.go:439-442);
* a file the staging cannot take (a read error, a short read) is zeroed, so
  IsBinary skips it and no stale bytes of an earlier batch are scanned.

Image layers take walker.analyze_layers (one GPU call per layer) in the
tagged build; a layer file that reaches this analyzer anyway (its FileInfo is
a tar header, walker.FileInfo) is analyzed per file.
"""
from __future__ import annotations

import os
import re
import sys
import threading
from concurrent.futures import ThreadPoolExecutor, wait
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from . import _native as N
from . import secret as S
from .types import Secret

SKIP_FILES = ["go.mod", "go.sum", "package-lock.json", "yarn.lock", "pnpm-lock.yaml", "Pipfile.lock",
              "Gemfile.lock"]
SKIP_DIRS = [".git", "node_modules"]
SKIP_EXTS = [".jpg", ".png", ".gif", ".doc", ".pdf", ".bin", ".svg", ".socket", ".deb", ".rpm", ".zip",
             ".gz", ".gzip", ".tar", ".pyc"]

TYPE = "secret"
VERSION = 1


def is_binary(head: bytes, size: int) -> bool:
    """utils.IsBinary: any control byte in the first min(size,300) bytes."""
    for b in head[:min(size, 300)]:
        if b < 7 or b == 11 or 13 < b < 27 or 27 < b < 0x20 or b == 0x7F:
            return True
    return False


def _go_ext(name: str) -> str:
    """filepath.Ext."""
    for i in range(len(name) - 1, -1, -1):
        if name[i] == "/":
            break
        if name[i] == ".":
            return name[i:]
    return ""


def _log(msg: str) -> None:
    print(f"secret: {msg}", file=sys.stderr)


# ------------------------------------------------------- analyzer inputs --

class FsFileInfo:
    """os.FileInfo of a walked local file (walker/fs.go:65: d.Info()).  Its
    identity is the object -- the pointer the Go value holds -- and `real` the
    underlying file (what os.SameFile compares)."""
    __slots__ = ("name", "size", "is_dir", "real")

    def __init__(self, name: str, size: int, is_dir: bool = False, real: Optional[str] = None):
        self.name, self.size, self.is_dir, self.real = name, size, is_dir, real


def _size(info) -> int:
    return info if isinstance(info, int) else info.size


@dataclass
class AnalyzerOptions:
    """analyzer.AnalyzerOptions: the fields this path reads."""
    config_path: str = ""                 # SecretScannerOption.ConfigPath
    disabled_analyzers: Sequence[str] = ()
    file_patterns: Sequence[str] = ()     # "type:regex" (analyzer.go:325-343)
    device: Optional[int] = None


@dataclass
class AnalysisInput:
    """analyzer.AnalysisInput (analyzer.go:133-140); `content` is a binary
    file object (xio.ReadSeekerAt)."""
    dir: str
    file_path: str
    info: object
    content: object


@dataclass
class Application:
    """types.Application: what the post-analysis filter reads."""
    type: str
    file_path: str
    library_paths: List[str] = field(default_factory=list)  # Libraries[].FilePath


@dataclass
class AnalysisResult:
    """analyzer.AnalysisResult (analyzer.go:152-173), the fields this path uses."""
    secrets: List[Secret] = field(default_factory=list)
    applications: List[Application] = field(default_factory=list)
    system_installed_files: List[str] = field(default_factory=list)

    def __post_init__(self):
        self._m = threading.Lock()

    def merge(self, new: Optional["AnalysisResult"]) -> None:
        """Merge (analyzer.go:245-295)."""
        if new is None:
            return
        with self._m:
            self.applications += new.applications
            self.secrets += new.secrets
            self.system_installed_files += new.system_installed_files

    def sort(self) -> None:
        """Sort (analyzer.go:218-229) for secrets."""
        self.applications.sort(key=lambda a: (a.file_path, a.type))
        self.secrets.sort(key=lambda s: s.FilePath)
        for sec in self.secrets:
            sec.Findings.sort(key=lambda f: (f.RuleID, f.StartLine))


# ------------------------------------------------------- secret analyzer --

class SecretAnalyzer:
    def __init__(self, scanner: Optional[S.Scanner] = None, config_path: str = ""):
        self.scanner = scanner
        self.config_path = config_path

    def type(self) -> str:
        return TYPE

    def version(self) -> int:
        return VERSION

    def init(self, opts="", device: Optional[int] = None) -> None:
        """Init (secret.go:63-77): ParseConfig + NewScanner.  `opts` is an
        AnalyzerOptions (the Initializer call of analyzer.go:350-354) or the
        config path."""
        config_path = opts if isinstance(opts, str) else opts.config_path
        if not isinstance(opts, str) and device is None:
            device = opts.device
        if config_path == self.config_path and self.scanner is not None:
            return  # secret.go:64-68
        try:
            cfg = S.parse_config(config_path)
        except S.ConfigError as e:
            raise S.ConfigError(f"secret config error: {e}") from e
        self.scanner = S.new_scanner(cfg, device)
        self.config_path = config_path

    def required(self, file_path: str, info) -> bool:
        """Required (secret.go:115-153); `info` is a FileInfo or a size."""
        if _size(info) < 10:
            return False
        idx = file_path.rfind("/")
        d, name = (file_path[:idx + 1], file_path[idx + 1:]) if idx >= 0 else ("", file_path)
        dirs = d.split("/")
        if any(sd in dirs for sd in SKIP_DIRS):
            return False
        if name in SKIP_FILES:
            return False
        if os.path.basename(self.config_path) == file_path:
            return False
        if _go_ext(name) in SKIP_EXTS:
            return False
        if self.scanner.allow_path(file_path):
            return False
        return True

    def analyze(self, file_path: str, content: bytes, dir_: str = "") -> Optional[List[Secret]]:
        """Analyze (secret.go:79-113) for one file."""
        return self.analyze_batch([(file_path, content, dir_)])[0]

    def analyze_input(self, inp: AnalysisInput) -> Optional[AnalysisResult]:
        """Analyze(ctx, input) as AnalyzeFile calls it."""
        res = self.analyze(inp.file_path, _read_all(inp.content), inp.dir)
        return AnalysisResult(secrets=res) if res else None

    def analyze_batch(self, inputs: Sequence[Tuple[str, bytes, str]]) -> List[Optional[List[Secret]]]:
        """Batched Analyze (secret.go:79-113): the '/' prefix of secret.go:95-98
        on the path here; the IsBinary gate, '\r' deletion and Scan of every
        file in one GPU call (tsg_analyze)."""
        batch = [S.ScanArgs(path if dir_ != "" else "/" + path, content) for path, content, dir_ in inputs]
        out: List[Optional[List[Secret]]] = [None] * len(inputs)
        if batch:
            for i, res in enumerate(self.scanner.analyze_batch(batch)):
                if res is not None and res.Findings:
                    out[i] = [res]
        return out


def _read_all(content) -> bytes:
    return content if isinstance(content, (bytes, bytearray)) else content.read()


# ------------------------------------------------------- analyzer group --

class Registry:
    """The package-level analyzer maps (analyzer.go:93-107): analyzers by
    type, post-analyzer initialisers by type."""

    def __init__(self):
        self.analyzers: Dict[str, object] = {}
        self.post_analyzers: Dict[str, Callable[[AnalyzerOptions], object]] = {}

    def register_analyzer(self, a) -> None:
        if a.type() in self.analyzers:
            raise RuntimeError(f"Analyzer is registered twice: {a.type()}")
        self.analyzers[a.type()] = a

    def register_post_analyzer(self, t: str, init: Callable[[AnalyzerOptions], object]) -> None:
        if t in self.post_analyzers:
            raise RuntimeError(f"Analyzer is registered twice: {t}")
        self.post_analyzers[t] = init


class MapFS:
    """mapfs.FS of one post-analyzer: virtual path -> underlying path."""

    def __init__(self, files: Optional[Dict[str, str]] = None):
        self.files: Dict[str, str] = dict(files or {})

    def filter(self, skipped: Sequence[str]) -> "MapFS":
        """Filter (mapfs/fs.go:69-77): a new FS without the skipped paths."""
        if not skipped:
            return self
        sk = set(skipped)
        return MapFS({p: r for p, r in self.files.items() if p not in sk})

    def walk(self):
        """fs.WalkDir order (lexical by path element)."""
        return sorted(self.files.items(), key=lambda kv: kv[0].split("/"))


class CompositeFS:
    """CompositeFS (analyzer/fs.go): one MapFS per post-analyzer type, made
    on the first link of that type (Get is false for a type nothing linked)."""

    def __init__(self):
        self.files: Dict[str, MapFS] = {}
        self._m = threading.Lock()

    def create_link(self, types: Sequence[str], root: str, vpath: str, real: str) -> None:
        with self._m:
            for t in types:
                self.files.setdefault(t, MapFS()).files[vpath] = real

    def get(self, t: str) -> Optional[MapFS]:
        return self.files.get(t)


class AnalyzerGroup:
    """AnalyzerGroup (analyzer.go:122-127, 315-370, 396-503)."""

    def __init__(self):
        self.analyzers: List[object] = []
        self.post_analyzers: List[object] = []
        self.file_patterns: Dict[str, List[re.Pattern]] = {}

    @classmethod
    def new(cls, registry: Registry, opts: AnalyzerOptions) -> "AnalyzerGroup":
        """NewAnalyzerGroup (analyzer.go:315-370): an analyzer is skipped when
        disabled BEFORE its Init; a post-analyzer's initialiser runs first and
        the disabled check comes after it (:358-365)."""
        g = cls()
        for p in opts.file_patterns:
            t, sep, pat = p.partition(":")
            if not sep:
                raise ValueError(f"invalid file pattern ({p})")
            g.file_patterns.setdefault(t, []).append(re.compile(pat))
        for t, a in registry.analyzers.items():
            if t in opts.disabled_analyzers:
                continue
            if hasattr(a, "init"):
                a.init(opts)
            g.analyzers.append(a)
        for t, init in registry.post_analyzers.items():
            a = init(opts)
            if t in opts.disabled_analyzers:
                continue
            g.post_analyzers.append(a)
        return g

    def _pattern(self, t: str, path: str) -> bool:
        return any(r.search(path) for r in self.file_patterns.get(t, ()))

    def analyze_file(self, pool: ThreadPoolExecutor, pending: list, result: AnalysisResult, dir_: str,
                     file_path: str, info, opener, disabled: Sequence[str] = ()) -> None:
        """AnalyzeFile (analyzer.go:396-448): per analyzer, Required (or a
        file pattern) then Analyze in a goroutine (here: the pool) whose error
        is logged and dropped."""
        if info.is_dir:
            return
        clean = file_path.lstrip("/")
        for a in self.analyzers:
            if a.type() in disabled:
                continue
            if not self._pattern(a.type(), clean) and not a.required(clean, info):
                continue
            try:
                rc = opener()
            except PermissionError:
                break  # analyzer.go:415-417
            pending.append(pool.submit(self._analyze, a, result, AnalysisInput(dir_, file_path, info, rc)))

    @staticmethod
    def _analyze(a, result: AnalysisResult, inp: AnalysisInput) -> None:
        try:
            ret = a.analyze_input(inp)
        except Exception as e:  # noqa: BLE001 -- analyzer.go:439-442
            _log(f"Analysis error: {e}")
            return
        finally:
            close = getattr(inp.content, "close", None)
            if close:
                close()
        result.merge(ret)

    def required_post_analyzers(self, file_path: str, info) -> List[str]:
        """RequiredPostAnalyzers (analyzer.go:451-462)."""
        if info.is_dir:
            return []
        return [a.type() for a in self.post_analyzers if self._pattern(a.type(), file_path) or a.required(file_path, info)]

    def post_analyze(self, composite: CompositeFS, result: AnalysisResult) -> None:
        """PostAnalyze (analyzer.go:468-503): each post-analyzer gets its FS
        minus SystemInstalledFiles and every Application's (and library's)
        FilePath; an error aborts ("post analysis error")."""
        for a in self.post_analyzers:
            fsys = composite.get(a.type())
            if fsys is None:
                continue
            skipped = list(result.system_installed_files)
            for app in result.applications:
                skipped.append(app.file_path)
                skipped += [p for p in app.library_paths if p]
            res = a.post_analyze(fsys.filter(skipped))
            result.merge(res)


def walk_local(root: str):
    """walker.FS.Walk (walker/fs.go:24-75) without skip options: regular
    files as (slash relative path, FsFileInfo), filepath.WalkDir order."""
    def rec(rel):
        full = os.path.join(root, rel) if rel else root
        for name in sorted(os.listdir(full)):
            p = f"{rel}/{name}" if rel else name
            fp = os.path.join(root, p)
            if os.path.isdir(fp) and not os.path.islink(fp):
                yield from rec(p)
            elif os.path.isfile(fp) and not os.path.islink(fp):
                yield p, FsFileInfo(name, os.path.getsize(fp), real=fp)
    yield from rec("")


def inspect_local(root: str, group: AnalyzerGroup, parallel: int = 5) -> AnalysisResult:
    """Artifact.Inspect of a filesystem artifact (artifact/local/fs.go:70-125):
    AnalyzeFile + RequiredPostAnalyzers/CreateLink per walked file, wait for
    every Analyze, PostAnalyze, Sort."""
    result = AnalysisResult()
    composite = CompositeFS()
    root = root.rstrip("/") or "/"
    with ThreadPoolExecutor(max_workers=max(1, parallel)) as pool:
        pending: list = []
        for rel, info in walk_local(root):
            group.analyze_file(pool, pending, result, root, rel, info,
                               lambda fp=info.real: open(fp, "rb"))
            types = group.required_post_analyzers(rel, info)
            if types:
                composite.create_link(types, root, rel, info.real)
        wait(pending)  # wg.Wait() (fs.go:112-113)
    group.post_analyze(composite, result)
    result.sort()
    return result


# ---------------------------------------------- the tagged build's analyzer --

GPU_BATCH_BYTES = 512 << 20  # --secret-gpu-batch-bytes


class _Staged:
    """The process's staging buffer and what is in it: one entry per
    reserved slot (FileInfo, scan path, Analyze's path and dir, the slot) and
    the count of slots still being filled (sync.WaitGroup in Go)."""

    def __init__(self, batch: "S.Batch"):
        self.batch = batch
        self.entries: List[tuple] = []
        self.filling = 0
        self.cv = threading.Condition()

    def wait_fills(self) -> None:
        with self.cv:
            while self.filling:
                self.cv.wait()

    def fill_done(self) -> None:
        with self.cv:
            self.filling -= 1
            self.cv.notify_all()


class GPUSecretAnalyzer(SecretAnalyzer):
    """gpuSecrets (secret_mi355x.go): the process-wide secret analyzer of the
    tagged build, registered both as the per-file analyzer and (through
    post_analyzer_init) as the post-analyzer that closes each walk.

    `go_analyze(file_path, raw, dir)`: Trivy's own per-file
    SecretAnalyzer.Analyze, the path a host without a usable GPU, a failed
    batch or a tar-header file takes in the Go build (the pure-Go Scanner);
    None here means the GPU analyzes such files one at a time instead."""

    def __init__(self, batch_bytes: int = GPU_BATCH_BYTES,
                 go_analyze: Optional[Callable[[str, bytes, str], Optional[List]]] = None):
        super().__init__()
        self.batch_bytes = batch_bytes
        self.go_analyze = go_analyze
        self._mu = threading.Lock()        # staging reservation and batch runs
        self._st: Optional[_Staged] = None
        self._ready = False                # lazy backend probed
        self._gpu_err: Optional[Exception] = None
        self._results: Dict[int, Tuple[object, Optional[Secret]]] = {}  # id(info) -> (info, secret)
        self._rmu = threading.Lock()

    # -- Initializer: ParseConfig + NewScanner compile the ruleset (host only);
    # no engine, no staging: those are made at the first Analyze
    def init(self, opts="", device: Optional[int] = None) -> None:
        prev = self.scanner
        super().init(opts, device)
        if self.scanner is not prev:
            with self._mu:
                if self._st is not None:
                    self._st.batch.close()
                self._st, self._ready, self._gpu_err = None, False, None

    def _backend(self) -> bool:
        """The engine and the staging buffer, made once (sync.Once in Go);
        False when the host has no usable GPU (the per-file path then)."""
        if not self._ready:
            try:
                self._st = _Staged(self.scanner.new_batch(self.batch_bytes))
            except N.EngineError as e:
                self._gpu_err = e
                _log(f"mi355x backend unavailable, Trivy's Scan per file: {e}")
            self._ready = True
        return self._gpu_err is None

    def _per_file(self, inp: AnalysisInput) -> Optional[AnalysisResult]:
        raw = _read_all(inp.content)
        if self.go_analyze is not None:
            res = self.go_analyze(inp.file_path, raw, inp.dir)
        else:
            res = self.analyze(inp.file_path, raw, inp.dir)
        return AnalysisResult(secrets=list(res)) if res else None

    def analyze_input(self, inp: AnalysisInput) -> Optional[AnalysisResult]:
        """Analyze: stage the file; the results come back through PostAnalyze."""
        info = inp.info
        with self._mu:
            gpu = self._backend()
        if not gpu or not isinstance(info, FsFileInfo):
            return self._per_file(inp)  # no GPU, or a tar-header file (image layer)
        f = inp.content
        head = f.read(300)  # utils.IsBinary (utils.go:77-95), then back to the start
        if is_binary(head, info.size):
            return None
        f.seek(0)
        path = inp.file_path if inp.dir != "" else "/" + inp.file_path
        size = info.size
        with self._mu:
            st = self._st
            dst = st.batch.reserve(path, size)
            if dst is None and len(st.batch):
                self._run_locked(st)  # full: this Analyze runs the batch
                dst = st.batch.reserve(path, size)
            if dst is not None:
                st.entries.append((info, path, inp.file_path, inp.dir, dst))
                with st.cv:
                    st.filling += 1
        if dst is None:  # larger than the whole staging buffer: this file alone
            raw = f.read()
            out = self.scanner.analyze_batch([S.ScanArgs(path, raw)])[0]
            self._store(info, out)
            return None
        try:
            n = f.readinto(dst) if size else 0
            if n != size:
                raise OSError(f"short read ({n} of {size} bytes)")
        except OSError:
            # the slot must not keep an earlier batch's bytes: NULs make
            # IsBinary skip it, as the reference skips a file it cannot read
            dst[:] = bytes(size)
            raise
        finally:
            st.fill_done()
        return None

    def _run_locked(self, st: _Staged) -> None:
        """Analyze the staged files (caller holds _mu): wait for the slots
        still being filled, one tsg_analyze_staged; a failed batch is
        re-scanned file by file from the staged bytes."""
        st.wait_fills()
        entries, st.entries = st.entries, []
        try:
            out = st.batch.analyze()
        except N.EngineError as e:
            _log(f"GPU batch of {len(entries)} files failed ({e}); scanning them one by one")
            out = []
            for info, path, fpath, d, dst in entries:
                raw = bytes(dst)
                try:
                    if self.go_analyze is not None:
                        r = self.go_analyze(fpath, raw, d)
                        out.append(r[0] if r else None)
                    else:
                        out.append(self.scanner.analyze_batch([S.ScanArgs(path, raw)])[0])
                except Exception as e2:  # noqa: BLE001 -- the file's error is dropped (analyzer.go:439-442)
                    _log(f"Analysis error: {fpath}: {e2}")
                    out.append(None)
            st.batch.reset()
        for (info, *_), res in zip(entries, out):
            self._store(info, res)

    def _store(self, info, res: Optional[Secret]) -> None:
        with self._rmu:
            self._results[id(info)] = (info, res if res is not None and res.Findings else None)

    def _take(self, info) -> Optional[Secret]:
        with self._rmu:
            got = self._results.pop(id(info), None)
        return None if got is None else got[1]

    def flush(self) -> None:
        with self._mu:
            if self._st is not None and len(self._st.batch):
                self._run_locked(self._st)

    # -- the post-analyzer side: one per AnalyzerGroup (analyzer.go:358-366)
    def post_analyzer_init(self, opts: AnalyzerOptions) -> "_WalkCloser":
        return _WalkCloser(self)


class _WalkCloser:
    """The tagged build's secret post-analyzer: Required records the walk's
    files; PostAnalyze analyzes what is still staged and returns the results
    of exactly those files (and of the files a --file-patterns match linked
    without Required, found by os.SameFile)."""

    def __init__(self, owner: GPUSecretAnalyzer):
        self.owner = owner
        self.infos: List[object] = []
        self._m = threading.Lock()

    def type(self) -> str:
        return TYPE

    def version(self) -> int:
        return VERSION

    def required(self, file_path: str, info) -> bool:
        ok = self.owner.required(file_path, info)
        if ok:
            with self._m:
                self.infos.append(info)
        return ok

    def post_analyze(self, fsys: MapFS) -> Optional[AnalysisResult]:
        own = self.owner
        own.flush()
        secrets = []
        mine = {id(i) for i in self.infos}
        for info in self.infos:
            s = own._take(info)
            if s is not None:
                secrets.append(s)
        reals = {os.path.realpath(r) for _, r in fsys.walk()}
        with own._rmu:
            extra = [k for k, (info, _) in own._results.items()
                     if k not in mine and isinstance(info, FsFileInfo) and info.real
                     and os.path.realpath(info.real) in reals]
        for k in extra:
            with own._rmu:
                _, s = own._results.pop(k)
            if s is not None:
                secrets.append(s)
        self.infos = []
        return AnalysisResult(secrets=secrets) if secrets else None


def register_gpu_secret(registry: Registry, batch_bytes: int = GPU_BATCH_BYTES,
                        go_analyze=None) -> GPUSecretAnalyzer:
    """secret_mi355x.go init(): the one process-wide analyzer, registered as
    the per-file analyzer and as the post-analyzer of the same type."""
    a = GPUSecretAnalyzer(batch_bytes, go_analyze)
    registry.register_analyzer(a)
    registry.register_post_analyzer(TYPE, a.post_analyzer_init)
    return a
