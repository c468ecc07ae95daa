"""Mirror of the drop-in boundary, Trivy's SecretAnalyzer
(pkg/fanal/analyzer/secret/secret.go:28-153) and utils.IsBinary
(pkg/fanal/utils/utils.go:77-95), with a batched analyze for the GPU, and
the post-analyzer hook of the tagged Go build
(integration/go/pkg/fanal/analyzer/secret/secret_mi355x.go), mirrored line
for line by SecretPostAnalyzer.
"""
from __future__ import annotations

import os
import sys
from typing import List, Optional, Sequence, Tuple

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


class SecretAnalyzer:
    def __init__(self, scanner: Optional[S.Scanner] = None, config_path: str = ""):
        self.scanner = scanner
        self.config_path = config_path

    def type(self) -> str:
        return TYPE

    def version(self) -> int:
        return VERSION

    def init(self, config_path: str = "", device: Optional[int] = None) -> None:
        """Init (secret.go:63-77): ParseConfig + NewScanner."""
        try:
            cfg = S.parse_config(config_path)
        except S.ConfigError as e:
            raise S.ConfigError(f"secret config error: {e}") from e
        self.scanner = S.new_scanner(cfg, device)
        self.config_path = config_path

    def required(self, file_path: str, size: int) -> bool:
        """Required (secret.go:115-153)."""
        if size < 10:
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


GPU_BATCH_BYTES = 512 << 20  # --secret-gpu-batch-bytes


class SecretPostAnalyzer:
    """The tagged build's secret analyzer (secret_mi355x.go): registered as a
    PostAnalyzer (analyzer.go:78-82, RegisterPostAnalyzer :102-107), so the
    artifact walk only calls Required per file and links the required files
    into the post-analyzer FS (artifact/local/fs.go:100-106); PostAnalyze then
    reads every file straight into GPU staging and runs Analyze's per-file
    work (IsBinary, '\r' strip, Scan) batch by batch.  Paths are the FS's
    relative paths: a filesystem artifact calls Analyze with Dir = the scan
    root, so no '/' prefix (secret.go:95-98); image layers take
    walker.analyze_layers instead."""

    def __init__(self, analyzer: SecretAnalyzer, batch_bytes: int = GPU_BATCH_BYTES):
        self.analyzer = analyzer
        self.batch_bytes = batch_bytes

    def type(self) -> str:
        return TYPE

    def version(self) -> int:
        return VERSION

    def required(self, file_path: str, size: int) -> bool:
        return self.analyzer.required(file_path, size)

    def post_analyze(self, root: str) -> Optional[List[Secret]]:
        """PostAnalyze over the FS rooted at `root` (fs.WalkDir order:
        lexical per directory).  Returns AnalysisResult.Secrets (None when no
        file has findings)."""
        secrets: List[Secret] = []
        with self.analyzer.scanner.new_batch(self.batch_bytes) as batch:
            def flush():
                if len(batch) == 0:
                    return
                for s in batch.analyze():
                    if s is not None and s.Findings:
                        secrets.append(s)

            for path, size in _walk_dir(root):
                def fill(dst, p=path):
                    try:
                        with open(os.path.join(root, p), "rb") as f:
                            n = f.readinto(dst)
                        if n != len(dst):
                            raise OSError("short read")
                    except OSError as e:
                        # Analyze's read error skips the file (analyzer.go:430-434 logs it):
                        # NUL bytes make IsBinary skip it the same way
                        dst[:] = bytes(len(dst))
                        print(f"secret: read error {p}: {e}", file=sys.stderr)

                if batch.add(path, size, fill):
                    continue
                flush()
                if not batch.add(path, size, fill):  # larger than the whole staging: one file alone
                    with open(os.path.join(root, path), "rb") as f:
                        res = self.analyzer.analyze_batch([(path, f.read(), root)])[0]
                    if res:
                        secrets.extend(res)
            flush()
        return secrets or None


def _walk_dir(root: str):
    """fs.WalkDir(fsys, ".") regular files as (slash path, size), lexical order."""
    def rec(rel):
        full = os.path.join(root, rel) if rel else root
        for name in sorted(os.listdir(full)):
            p = f"{rel}/{name}" if rel else name
            fp = os.path.join(root, p)
            if os.path.isdir(fp) and not os.path.islink(fp):
                yield from rec(p)
            elif os.path.isfile(fp):
                yield p, os.path.getsize(fp)
    yield from rec("")
