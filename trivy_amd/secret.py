"""Host-side mirror of Trivy's secret engine API, backed by the MI355X engine.

Mirrors pkg/fanal/secret/scanner.go:
  * Config / Rule / AllowRule / ExcludeBlock ............ scanner.go:28-95,191-221
  * parse_config (ParseConfig) / convert_severity ........ scanner.go:272-313
  * new_scanner (NewScanner) ............................. scanner.go:315-359
  * Scanner.scan (Scan) / ScanArgs ....................... scanner.go:361-452
plus Scanner.scan_batch, the batched entry the GPU needs (many files per
launch).  Every byte of content is scanned by the HIP
kernels in csrc/engine.hip; this module only marshals rules and results.
"""
from __future__ import annotations

import ctypes
import dataclasses
import json
import os
import threading
from typing import List, Optional, Sequence

import yaml

from . import _native as N
from .types import Code, Line, Secret, SecretFinding

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "builtin_rules.json")


class ConfigError(ValueError):
    pass


@dataclasses.dataclass
class AllowRule:
    id: str = ""
    description: str = ""
    regex: Optional[str] = None
    path: Optional[str] = None


@dataclasses.dataclass
class ExcludeBlock:
    description: str = ""
    regexes: List[str] = dataclasses.field(default_factory=list)


@dataclasses.dataclass
class Rule:
    id: str = ""
    category: str = ""
    title: str = ""
    severity: str = ""
    regex: Optional[str] = None
    keywords: List[str] = dataclasses.field(default_factory=list)
    path: Optional[str] = None
    allow_rules: List[AllowRule] = dataclasses.field(default_factory=list)
    exclude_block: ExcludeBlock = dataclasses.field(default_factory=ExcludeBlock)
    secret_group_name: str = ""


@dataclasses.dataclass
class Config:
    enable_builtin_rule_ids: List[str] = dataclasses.field(default_factory=list)
    disable_rule_ids: List[str] = dataclasses.field(default_factory=list)
    disable_allow_rule_ids: List[str] = dataclasses.field(default_factory=list)
    custom_rules: List[Rule] = dataclasses.field(default_factory=list)
    custom_allow_rules: List[AllowRule] = dataclasses.field(default_factory=list)
    exclude_block: ExcludeBlock = dataclasses.field(default_factory=ExcludeBlock)


@dataclasses.dataclass
class ScanArgs:
    file_path: str
    content: bytes


# ---------------------------------------------------------------- builtin --

def _load_builtin():
    with open(_DATA) as fh:
        d = json.load(fh)
    rules = [Rule(id=r["id"], category=r["category"], title=r["title"], severity=r["severity"],
                  regex=r["regex"], keywords=list(r["keywords"]), secret_group_name=r["secret_group_name"])
             for r in d["rules"]]
    allows = [AllowRule(id=a["id"], description=a["description"], regex=a["regex"], path=a["path"])
              for a in d["allow_rules"]]
    return rules, allows


BUILTIN_RULES, BUILTIN_ALLOW_RULES = _load_builtin()


# ----------------------------------------------------------------- config --

def _validate_regex(src, what):
    """regexp.Compile at YAML decode time (scanner.go:70-82)."""
    if src is None:
        return None
    src = str(src)
    m = ctypes.c_int()
    rc = N.lib.tsg_regex_match(src.encode(), b"", 0, ctypes.byref(m))
    if rc == N.TSG_ERR_REGEX:
        raise ConfigError(f"secrets config decode error: regexp compile error: {N.lib.tsg_last_error().decode()}")
    if rc == N.TSG_ERR_UNSUPPORTED:
        raise ConfigError(N.lib.tsg_last_error().decode())
    return src


def convert_severity(severity) -> str:
    """scanner.go:305-313."""
    s = "" if severity is None else str(severity)
    if s.lower() in ("low", "medium", "high", "critical", "unknown"):
        return s.upper()
    return "UNKNOWN"


def _allow_rules(lst):
    out = []
    for a in lst or []:
        out.append(AllowRule(id=str(a.get("id") or ""), description=str(a.get("description") or ""),
                             regex=_validate_regex(a.get("regex"), "allow regex"),
                             path=_validate_regex(a.get("path"), "allow path")))
    return out


def _exclude_block(d):
    d = d or {}
    return ExcludeBlock(description=str(d.get("description") or ""),
                        regexes=[_validate_regex(x, "exclude") for x in (d.get("regexes") or [])])


def parse_config(config_path: str) -> Optional[Config]:
    """ParseConfig (scanner.go:272-302): None for "" or a missing file."""
    if not config_path:
        return None
    if not os.path.exists(config_path):
        return None
    with open(config_path) as fh:
        try:
            raw = yaml.safe_load(fh) or {}
        except yaml.YAMLError as e:
            raise ConfigError(f"secrets config decode error: {e}") from e
    cfg = Config(
        enable_builtin_rule_ids=[str(x) for x in raw.get("enable-builtin-rules") or []],
        disable_rule_ids=[str(x) for x in raw.get("disable-rules") or []],
        disable_allow_rule_ids=[str(x) for x in raw.get("disable-allow-rules") or []],
        custom_allow_rules=_allow_rules(raw.get("allow-rules")),
        exclude_block=_exclude_block(raw.get("exclude-block")),
    )
    for r in raw.get("rules") or []:
        cfg.custom_rules.append(Rule(
            id=str(r.get("id") or ""), category=str(r.get("category") or ""), title=str(r.get("title") or ""),
            severity=convert_severity(r.get("severity")), regex=_validate_regex(r.get("regex"), "regex"),
            keywords=[str(k) for k in r.get("keywords") or []], path=_validate_regex(r.get("path"), "path"),
            allow_rules=_allow_rules(r.get("allow-rules")), exclude_block=_exclude_block(r.get("exclude-block")),
            secret_group_name=str(r.get("secret-group-name") or "")))
    return cfg


# ----------------------------------------------------------------- engine --

_ENGINES = {}
_ENGINE_LOCK = threading.Lock()


def default_device() -> int:
    return int(os.environ.get("TSG_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def get_engine(device: Optional[int] = None):
    """One tsg_engine (HIP stream + device buffers) per GPU per process."""
    dev = default_device() if device is None else device
    with _ENGINE_LOCK:
        if dev not in _ENGINES:
            h = ctypes.c_void_p()
            N.check(N.lib.tsg_engine_create(dev, ctypes.byref(h)))
            _ENGINES[dev] = h
        return _ENGINES[dev]


_EXTRA_ENGINES = {}


def get_engines(device: Optional[int] = None, n: int = 2):
    """n engines on one GPU (the first is get_engine's): independent streams
    and buffers, so one engine's host-to-device staging overlaps another's
    pipeline (analyze_layers)."""
    dev = default_device() if device is None else device
    first = get_engine(dev)
    with _ENGINE_LOCK:
        extra = _EXTRA_ENGINES.setdefault(dev, [])
        while len(extra) < n - 1:
            h = ctypes.c_void_p()
            N.check(N.lib.tsg_engine_create(dev, ctypes.byref(h)))
            extra.append(h)
        return [first] + extra[: n - 1]


class _CompiledRuleSet:
    def __init__(self, rules: Sequence[Rule], allow_rules: Sequence[AllowRule], exclude: ExcludeBlock):
        keep = []
        enc = lambda s: None if s is None else s.encode("utf-8", "surrogateescape")
        crules = (N.RuleC * max(1, len(rules)))()
        for i, r in enumerate(rules):
            kws = (ctypes.c_char_p * max(1, len(r.keywords)))(*[enc(k) for k in r.keywords])
            ars = (N.AllowRuleC * max(1, len(r.allow_rules)))()
            for j, a in enumerate(r.allow_rules):
                ars[j].id, ars[j].regex, ars[j].path = enc(a.id), enc(a.regex), enc(a.path)
            exs = (ctypes.c_char_p * max(1, len(r.exclude_block.regexes)))(
                *[enc(x) for x in r.exclude_block.regexes])
            keep += [kws, ars, exs]
            c = crules[i]
            c.id, c.regex, c.path = enc(r.id), enc(r.regex), enc(r.path)
            c.keywords, c.n_keywords = kws, len(r.keywords)
            c.secret_group_name = enc(r.secret_group_name)
            c.allow_rules, c.n_allow_rules = ars, len(r.allow_rules)
            c.exclude_regexes, c.n_exclude_regexes = exs, len(r.exclude_block.regexes)
        gar = (N.AllowRuleC * max(1, len(allow_rules)))()
        for j, a in enumerate(allow_rules):
            gar[j].id, gar[j].regex, gar[j].path = enc(a.id), enc(a.regex), enc(a.path)
        gex = (ctypes.c_char_p * max(1, len(exclude.regexes)))(*[enc(x) for x in exclude.regexes])
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(1024)
        rc = N.lib.tsg_ruleset_compile(crules, len(rules), gar, len(allow_rules), gex, len(exclude.regexes),
                                       ctypes.byref(h), err, 1024)
        if rc != N.TSG_OK:
            raise N.EngineError(rc, err.value.decode("utf-8", "replace"))
        self.handle = h

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            N.lib.tsg_ruleset_free(h)
            self.handle = None


def _s(ptr, n) -> str:
    return ctypes.string_at(ptr, n).decode("utf-8", "surrogateescape") if n else ""


class Scanner:
    """NewScanner result; Scan/scan_batch run on the MI355X."""

    def __init__(self, rules: List[Rule], allow_rules: List[AllowRule], exclude_block: ExcludeBlock,
                 device: Optional[int] = None):
        self.rules = rules
        self.allow_rules = allow_rules
        self.exclude_block = exclude_block
        self.device = device
        self._rs = _CompiledRuleSet(rules, allow_rules, exclude_block)
        self.last_timings_ms: List[float] = []

    # Global.AllowPath (scanner.go:55-58, 200-207): per-file host check.
    def allow_path(self, path: str) -> bool:
        """Global AllowPath (scanner.go:200-207) with the compiled ruleset's regexes."""
        p = path.encode("utf-8", "surrogateescape")
        m = ctypes.c_int()
        N.check(N.lib.tsg_ruleset_allow_path(self._rs.handle, p, len(p), ctypes.byref(m)))
        return bool(m.value)

    def scan(self, args: ScanArgs) -> Secret:
        return self.scan_batch([args])[0]

    def scan_batch(self, batch: Sequence[ScanArgs]) -> List[Secret]:
        return self._run(N.lib.tsg_scan, batch)

    def scan_batch_device(self, batch: Sequence[ScanArgs]) -> List[Secret]:
        """Scan through tsg_scan_device: the batch is packed into HBM first
        (content + one NUL separator per file, the layout include/
        trivy_secret_gpu.h documents) and the findings -- Match and Code
        included -- are built on the device.  Device memory comes from the HIP
        runtime the engine itself links (no second runtime in the process)."""
        import numpy as np

        get_engine(self.device)  # selects and initialises the device first
        n = len(batch)
        off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(np.array([len(a.content) + 1 for a in batch], dtype=np.uint64), out=off[1:])
        host = np.zeros(int(off[-1]) + 16, dtype=np.uint8)
        for i, a in enumerate(batch):
            host[int(off[i]):int(off[i]) + len(a.content)] = np.frombuffer(bytes(a.content), dtype=np.uint8)
        paths = [a.file_path.encode("utf-8", "surrogateescape") for a in batch]
        poff = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(np.array([len(x) for x in paths], dtype=np.uint64), out=poff[1:])
        pbuf = np.frombuffer(b"".join(paths) + b"\0" * 16, dtype=np.uint8)
        bufs = [N.DeviceBuffer(x) for x in (host, off, pbuf, poff)]
        try:
            res = ctypes.c_void_p()
            N.check(N.lib.tsg_scan_device(get_engine(self.device), self._rs.handle, *[b.ptr for b in bufs], n,
                                          ctypes.byref(res)))
            try:
                return self._convert(res, batch)
            finally:
                N.lib.tsg_result_free(res)
        finally:
            for b in bufs:
                b.free()

    # ---- byte-range split of one large file (tsg_scan_part_device /
    # tsg_scan_merge_device); trivy_amd.shard.scan_split drives it across ranks
    def part_halo(self):
        """(left, right): the bytes a part's view must hold around its range."""
        lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
        N.check(N.lib.tsg_part_halo(self._rs.handle, ctypes.byref(lo), ctypes.byref(hi)))
        return lo.value, hi.value

    def scan_part(self, view, text_base: int, own_lo: int, own_hi: int, file_len: int, file_path: str) -> bytes:
        """Scan pass over file bytes [own_lo, own_hi): `view` holds file bytes
        [text_base, text_base + len(view)) covering part_halo() around the
        range.  Returns the part's scan state (opaque bytes) for the owner."""
        import numpy as np

        get_engine(self.device)
        # + one readable byte after the view: a NUL, which only literals starting
        # past own_hi could touch (the next part owns those)
        host = np.zeros(len(view) + 1, dtype=np.uint8)
        host[:len(view)] = np.frombuffer(bytes(view), dtype=np.uint8)
        buf = N.DeviceBuffer(host)
        try:
            blob, n = ctypes.c_void_p(), ctypes.c_size_t()
            N.check(N.lib.tsg_scan_part_device(get_engine(self.device), self._rs.handle, buf.ptr, text_base, len(view),
                                               own_lo, own_hi, file_len, file_path.encode("utf-8", "surrogateescape"),
                                               ctypes.byref(blob), ctypes.byref(n)))
            try:
                return ctypes.string_at(blob, n.value)
            finally:
                N.lib.tsg_part_free(blob)
        finally:
            buf.free()

    def scan_merge(self, args: ScanArgs, parts: Sequence[bytes]) -> Secret:
        """The owner's side: the whole file in HBM + the parts' scan states ->
        the same Secret tsg_scan_device gives for the file."""
        import numpy as np

        get_engine(self.device)
        host = np.zeros(len(args.content) + 16, dtype=np.uint8)
        host[:len(args.content)] = np.frombuffer(bytes(args.content), dtype=np.uint8)
        buf = N.DeviceBuffer(host)
        keep = [ctypes.create_string_buffer(bytes(p), len(p)) for p in parts]
        ptrs = (ctypes.c_void_p * max(1, len(parts)))(*[ctypes.cast(k, ctypes.c_void_p) for k in keep])
        lens = (ctypes.c_size_t * max(1, len(parts)))(*[len(p) for p in parts])
        try:
            res = ctypes.c_void_p()
            N.check(N.lib.tsg_scan_merge_device(get_engine(self.device), self._rs.handle, buf.ptr, len(args.content),
                                                args.file_path.encode("utf-8", "surrogateescape"), ptrs, lens,
                                                len(parts), ctypes.byref(res)))
            try:
                return self._convert(res, [args])[0]
            finally:
                N.lib.tsg_result_free(res)
        finally:
            buf.free()

    def analyze_batch(self, batch: Sequence[ScanArgs]) -> List[Optional[Secret]]:
        """SecretAnalyzer.Analyze's per-file work on the GPU (tsg_analyze):
        IsBinary gate, '\r' deletion, Scan.  `content` is the raw file; None
        for binary files (secret.go:80-86)."""
        return self._run(N.lib.tsg_analyze, batch)

    def new_batch(self, capacity: int) -> "Batch":
        """A caller-filled staging batch (tsg_staging_*) for this scanner."""
        return Batch(self, capacity)

    def _run(self, fn, batch: Sequence[ScanArgs]):
        eng = get_engine(self.device)
        n = len(batch)
        files = (N.FileC * max(1, n))()
        keep = []
        for i, a in enumerate(batch):
            buf = ctypes.create_string_buffer(bytes(a.content), len(a.content)) if a.content else None
            keep.append(buf)
            files[i].data = ctypes.cast(buf, ctypes.c_void_p) if buf is not None else None
            files[i].len = len(a.content)
            files[i].path = a.file_path.encode("utf-8", "surrogateescape")
        res = ctypes.c_void_p()
        N.check(fn(eng, self._rs.handle, files, n, ctypes.byref(res)))
        try:
            return self._convert(res, batch)
        finally:
            N.lib.tsg_result_free(res)

    def _convert(self, res, batch) -> List[Secret]:
        tm = (ctypes.c_double * 16)()
        nt = ctypes.c_size_t()
        N.lib.tsg_result_timings(res, tm, 16, ctypes.byref(nt))
        self.last_timings_ms = [tm[i] for i in range(min(16, nt.value))]
        flags = N.lib.tsg_result_file_flags(res)
        out = []
        for i in range(len(batch)):  # batch[i] only where a FilePath is emitted (lazy batches)
            if flags[i] & N.TSG_FILE_BINARY:
                out.append(None)
                continue
            if flags[i] & N.TSG_FILE_PATH_ALLOWED:
                out.append(Secret(FilePath=batch[i].file_path))
                continue
            fp = ctypes.POINTER(N.FindingC)()
            k = N.lib.tsg_result_findings(res, i, ctypes.byref(fp))
            if k == 0:
                out.append(Secret())
                continue
            findings = []
            for j in range(k):
                f = fp[j]
                rule = self.rules[f.rule]
                lines = []
                for q in range(f.n_lines):
                    ln = f.lines[q]
                    txt = _s(ln.content, ln.content_len)
                    lines.append(Line(Number=ln.number, Content=txt, IsCause=bool(ln.is_cause),
                                      Highlighted=txt, FirstCause=bool(ln.first_cause),
                                      LastCause=bool(ln.last_cause)))
                findings.append(SecretFinding(
                    RuleID=rule.id, Category=rule.category, Severity=rule.severity or "UNKNOWN",
                    Title=rule.title, StartLine=f.start_line, EndLine=f.end_line,
                    Code=Code(Lines=lines), Match=_s(f.match, f.match_len)))
            out.append(Secret(FilePath=batch[i].file_path, Findings=findings))
        return out


class Batch:
    """Mirror of the Go backend's Batch (integration/go/pkg/fanal/secret/
    gpu_mi355x.go): files are read straight into a page-locked staging buffer
    (tsg_staging_add hands out where each file goes), then one call runs the
    whole batch -- tsg_analyze_staged (RAW files: IsBinary, '\r' strip, Scan)
    or tsg_scan_staged (CR-stripped content) -- and the staging is reset."""

    def __init__(self, scanner: Scanner, capacity: int):
        self.scanner = scanner
        self.handle = ctypes.c_void_p()
        get_engine(scanner.device)  # selects and initialises the device first
        N.check(N.lib.tsg_staging_create(capacity, ctypes.byref(self.handle)))
        self.paths: List[str] = []

    def __len__(self) -> int:
        return len(self.paths)

    def reserve(self, file_path: str, size: int) -> Optional[memoryview]:
        """Reserve `size` bytes for file_path (Batch.Reserve in Go): the
        writable slot (empty for size 0), or None when the staging has no room
        (run the batch and reserve again).  The caller fills the slot before
        the batch runs -- and zeroes it if it cannot (a slot keeps whatever an
        earlier batch left there)."""
        dst = ctypes.c_void_p()
        rc = N.lib.tsg_staging_add(self.handle, file_path.encode("utf-8", "surrogateescape"), size,
                                   ctypes.byref(dst))
        if rc == N.TSG_ERR_FULL:
            return None
        N.check(rc)
        self.paths.append(file_path)
        if not size:
            return memoryview(bytearray(0))
        return memoryview((ctypes.c_uint8 * size).from_address(dst.value)).cast("B")

    def add(self, file_path: str, size: int, fill) -> bool:
        """Reserve `size` bytes for file_path and let fill(dst) write them in
        place (dst: a writable memoryview of exactly `size` bytes).  False when
        the staging has no room (run the batch and add again).  A fill that
        raises leaves the slot zeroed (IsBinary then skips the file) and the
        error propagates."""
        dst = self.reserve(file_path, size)
        if dst is None:
            return False
        if size:
            try:
                fill(dst)
            except BaseException:
                dst[:] = bytes(size)
                raise
        return True

    def reset(self) -> None:
        """Empty the batch without running it (tsg_staging_reset)."""
        N.lib.tsg_staging_reset(self.handle)
        self.paths = []

    def analyze(self) -> List[Optional[Secret]]:
        """tsg_analyze_staged; None for binary files (secret.go:80-86)."""
        return self._run(N.lib.tsg_analyze_staged)

    def scan(self) -> List[Secret]:
        return self._run(N.lib.tsg_scan_staged)

    def _run(self, fn):
        """One staged call; on success the batch is reset.  On an error the
        staged files stay (the caller may re-scan them from their slots, then
        reset)."""
        res = ctypes.c_void_p()
        N.check(fn(get_engine(self.scanner.device), self.scanner._rs.handle, self.handle, ctypes.byref(res)))
        try:
            return self.scanner._convert(res, [ScanArgs(p, b"") for p in self.paths])
        finally:
            N.lib.tsg_result_free(res)
            self.reset()

    def close(self) -> None:
        if self.handle:
            N.lib.tsg_staging_free(self.handle)
            self.handle = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()


def new_scanner(config: Optional[Config] = None, device: Optional[int] = None) -> Scanner:
    """NewScanner (scanner.go:315-359)."""
    if config is None:
        return Scanner(list(BUILTIN_RULES), list(BUILTIN_ALLOW_RULES), ExcludeBlock(), device)
    enabled = list(BUILTIN_RULES)
    if config.enable_builtin_rule_ids:
        enabled = [r for r in BUILTIN_RULES if r.id in config.enable_builtin_rule_ids]
    enabled += list(config.custom_rules)
    rules = [r for r in enabled if r.id not in config.disable_rule_ids]
    allows = list(BUILTIN_ALLOW_RULES) + list(config.custom_allow_rules)
    allows = [a for a in allows if a.id not in config.disable_allow_rule_ids]
    return Scanner(rules, allows, config.exclude_block, device)
