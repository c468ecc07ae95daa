"""CPU ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/secret_oracle.py's header).

Restates walker.LayerTar.Walk (pkg/fanal/walker/tar.go:35-117) and
walker.SkipPath/CleanSkipPaths (walk.go:28-53) with Python's stdlib
``tarfile`` (stream mode) as the tar reader, independent of the engine's
native header parser, and doublestar.Match (github.com/bmatcuk/doublestar/v4,
v4.6.1 per the reference's go.mod; not in the reference tree) restated by
translating a glob into a regular expression.

Pinning: the reference's own TestLayerTar_Walk cases over
pkg/fanal/walker/testdata/test.tar (copied to tests/golden/walker/test.tar):
opq dirs ["etc/"], whiteouts ["foo/foo"], SkipFiles/SkipDirs and the
analyze-error wrap.  Long names, PAX records, glob corner cases and malformed
archives are restatement-derived, not Go-verified.
"""
from __future__ import annotations

import io
import posixpath
import re
import tarfile
from typing import Callable, List, Sequence, Tuple


def go_path_clean(p: str) -> str:
    """path.Clean (Go).  posixpath.normpath keeps a leading '//' — Go does not."""
    if p == "":
        return "."
    rooted = p.startswith("/")
    parts: List[str] = []
    for e in p.split("/"):
        if e in ("", "."):
            continue
        if e == "..":
            if parts and parts[-1] != "..":
                parts.pop()
            elif not rooted:
                parts.append("..")
            continue
        parts.append(e)
    out = ("/" if rooted else "") + "/".join(parts)
    return out or "."


def _glob_to_regex(pat: str) -> str:
    """doublestar v4 glob -> regex.  Raises ValueError on a bad pattern."""
    out, i, n = [], 0, len(pat)
    depth = 0
    while i < n:
        c = pat[i]
        if c == "*":
            j = i
            while j < n and pat[j] == "*":
                j += 1
            whole = (i == 0 or pat[i - 1] == "/") and (j == n or pat[j] == "/") and j - i == 2
            if whole:
                if j == n:  # trailing '**': everything (and the dir itself via the '/' case)
                    out.append(".*")
                else:  # '**/': zero or more whole components
                    out.append("(?:[^/]*(?:/[^/]*)*/)?")
                    j += 1
            else:
                out.append("[^/]*")
            i = j
            continue
        if c == "/" and pat[i:] == "/**":
            out.append("(?:/.*)?")
            i = n
            continue
        if c == "?":
            out.append("[^/]")
        elif c == "[":
            j = i + 1
            neg = j < n and pat[j] in "!^"
            if neg:
                j += 1
            items, first = [], True
            while j < n and (first or pat[j] != "]"):
                first = False
                lo = pat[j]
                if lo == "\\" and j + 1 < n:
                    j += 1
                    lo = pat[j]
                j += 1
                hi = lo
                if j + 1 < n and pat[j] == "-" and pat[j + 1] != "]":
                    hi = pat[j + 1]
                    if hi == "\\" and j + 2 < n:
                        j += 1
                        hi = pat[j + 1]
                    j += 2
                items.append(re.escape(lo) + ("-" + re.escape(hi) if hi != lo else ""))
            if j >= n:
                raise ValueError("syntax error in pattern")
            body = "".join(items)
            out.append(f"(?![/])[^{body}]" if neg else f"(?![/])[{body}]")
            i = j
        elif c == "{":
            depth += 1
            out.append("(?:")
        elif c == "," and depth:
            out.append("|")
        elif c == "}" and depth:
            depth -= 1
            out.append(")")
        elif c == "\\" and i + 1 < n:
            i += 1
            out.append(re.escape(pat[i]))
        else:
            out.append(re.escape(c))
        i += 1
    if depth:
        raise ValueError("syntax error in pattern")
    return "".join(out)


def doublestar_match(pattern: str, path: str) -> bool:
    return re.fullmatch(_glob_to_regex(pattern), path, re.S) is not None


def clean_skip_paths(paths: Sequence[str]) -> List[str]:  # walk.go:30-35
    return [go_path_clean(p).lstrip("/") for p in paths]


def skip_path(path: str, patterns: Sequence[str]) -> bool:  # walk.go:39-53
    path = path.lstrip("/")
    for pat in patterns:
        try:
            if doublestar_match(pat, path):
                return True
        except ValueError:
            return False
    return False


def _rel(base: str, target: str) -> str:
    """filepath.Rel for clean relative paths (lexical)."""
    b = [] if base == "." else base.split("/")
    t = [] if target == "." else target.split("/")
    c = 0
    while c < len(b) and c < len(t) and b[c] == t[c]:
        c += 1
    parts = [".."] * (len(b) - c) + t[c:]
    return "/".join(parts) or "."


def under_skipped_dir(file_path: str, skip_dirs: Sequence[str]) -> bool:  # tar.go:106-117
    return any(not _rel(go_path_clean(d), file_path).startswith("../") for d in skip_dirs)


class WalkError(RuntimeError):
    pass


def walk(layer: bytes, analyze_fn: Callable[[str, int, bool, bytes], None],
         skip_files: Sequence[str] = (), skip_dirs: Sequence[str] = ()) -> Tuple[List[str], List[str]]:
    """LayerTar.Walk (tar.go:35-90): analyze_fn(path, size, is_dir, content)."""
    sf, sd = clean_skip_paths(skip_files), clean_skip_paths(skip_dirs)
    opq, wh, skipped = [], [], []
    try:
        tf = tarfile.open(fileobj=io.BytesIO(layer), mode="r|", ignore_zeros=False)
        members = iter(tf)
    except tarfile.ReadError as e:
        if len(layer) == 0:
            return [], []
        raise WalkError(f"failed to extract the archive: {e}") from e
    while True:
        try:
            m = next(members)
        except StopIteration:
            break
        except tarfile.TarError as e:
            raise WalkError(f"failed to extract the archive: {e}") from e
        fp = go_path_clean(m.name).lstrip("/")
        d, base = posixpath.split(fp)
        d = d + "/" if d else ""
        if base == ".wh..wh..opq":
            opq.append(d)
            continue
        if base.startswith(".wh."):
            wh.append(go_path_clean(d + base[4:]) if d or base[4:] else "")
            continue
        if m.isdir():
            if skip_path(fp, sd):
                skipped.append(fp)
                continue
        elif m.type in (tarfile.REGTYPE, tarfile.AREGTYPE):  # TypeCont falls to default
            if skip_path(fp, sf):
                continue
        else:
            continue
        if under_skipped_dir(fp, skipped):
            continue
        content = b"" if m.isdir() else tf.extractfile(m).read()
        try:
            analyze_fn(fp, 0 if m.isdir() else m.size, m.isdir(), content)
        except Exception as e:  # noqa: BLE001
            raise WalkError(f"failed to process the file: failed to analyze file: {e}") from e
    return opq, wh
