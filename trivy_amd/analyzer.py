"""Mirror of the drop-in boundary, Trivy's SecretAnalyzer
(pkg/fanal/analyzer/secret/secret.go:28-153) and utils.IsBinary
(pkg/fanal/utils/utils.go:77-95), with a batched analyze for the GPU.
"""
from __future__ import annotations

import os
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
