"""Mirror of the image-config secret analyzer, the second caller of the same
engine (pkg/fanal/analyzer/imgconf/secret/secret.go:26-62): the image's
v1.ConfigFile is rendered with Go's ``json.MarshalIndent(cfg, "  ", "")``
and scanned as one file named ``config.json`` on the MI355X.

The rendering restates encoding/json for the go-containerregistry
``v1.ConfigFile`` shape (a dependency absent from the reference tree): the
top-level fields in struct order with their omitempty rules, ``created``
always present (a zero ``v1.Time`` marshals as "0001-01-01T00:00:00Z"),
``rootfs`` always present; ``config`` in ``v1.Config`` struct order (every
field omitempty; keys the struct does not know follow in the caller's order),
its map fields (Labels, Volumes, ExposedPorts) with keys sorted as
encoding/json sorts map keys, and each ``history`` entry in ``v1.History``
order (author, created, created_by, comment, empty_layer) with ``created``
always present.  Parity is pinned by the reference's own test
(tests/golden/imgconf_cases.json); the config/history ordering beyond it is
restatement-derived (go-containerregistry v1 types, not in the reference tree).
"""
from __future__ import annotations

import json
from typing import Any, Optional

from . import secret as S
from .types import Secret

_ZERO_TIME = "0001-01-01T00:00:00Z"
# go-containerregistry pkg/v1 Config field order (all omitempty)
_CONFIG_ORDER = ["AttachStderr", "AttachStdin", "AttachStdout", "Cmd", "Healthcheck", "Domainname", "Entrypoint",
                 "Env", "Hostname", "Image", "Labels", "OnBuild", "OpenStdin", "StdinOnce", "Tty", "User", "Volumes",
                 "WorkingDir", "ExposedPorts", "ArgsEscaped", "NetworkDisabled", "MacAddress", "StopSignal", "Shell"]
_CONFIG_MAPS = {"Labels", "Volumes", "ExposedPorts"}
_HISTORY_ORDER = ["author", "created", "created_by", "comment", "empty_layer"]


def _go_config(c: dict) -> dict:
    """v1.Config in struct order, empty fields omitted, map keys sorted."""
    out = {}
    for k in _CONFIG_ORDER + [k for k in c if k not in _CONFIG_ORDER]:
        v = c.get(k)
        if _empty(v):
            continue
        out[k] = {m: v[m] for m in sorted(v)} if k in _CONFIG_MAPS and isinstance(v, dict) else v
    return out


def _go_history(h: dict) -> dict:
    """v1.History: `created` is a struct (never omitted), the rest omitempty."""
    out = {}
    for k in _HISTORY_ORDER:
        v = h.get(k)
        if k == "created":
            out[k] = v or _ZERO_TIME
        elif not _empty(v):
            out[k] = v
    return out


def _empty(v: Any) -> bool:
    return v is None or v is False or v == 0 or v == "" or v == [] or v == {}


def _go_string(s: str) -> str:
    # encoding/json escapes <, >, & (HTML-safe) and U+2028/9; ensure_ascii off
    out = json.dumps(s, ensure_ascii=False)
    return (out.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
            .replace("\u2028", "\\u2028").replace("\u2029", "\\u2029"))


def _render(v: Any, prefix: str, lines: list, head: str, tail: str) -> None:
    """Appends v's lines (MarshalIndent with indent "": every element on its
    own line, each line after the first carrying `prefix`)."""
    if isinstance(v, dict) and v:
        lines.append(head + "{")
        items = list(v.items())
        for i, (k, x) in enumerate(items):
            _render(x, prefix, lines, prefix + _go_string(k) + ": ", "," if i + 1 < len(items) else "")
        lines.append(prefix + "}" + tail)
    elif isinstance(v, list) and v:
        lines.append(head + "[")
        for i, x in enumerate(v):
            _render(x, prefix, lines, prefix, "," if i + 1 < len(v) else "")
        lines.append(prefix + "]" + tail)
    elif isinstance(v, dict):
        lines.append(head + "{}" + tail)
    elif isinstance(v, list):
        lines.append(head + "[]" + tail)
    elif v is None:
        lines.append(head + "null" + tail)
    elif isinstance(v, bool):
        lines.append(head + ("true" if v else "false") + tail)
    elif isinstance(v, (int, float)):
        lines.append(head + json.dumps(v) + tail)
    else:
        lines.append(head + _go_string(str(v)) + tail)


def marshal_config_file(cfg: dict) -> bytes:
    """json.MarshalIndent(v1.ConfigFile, "  ", "") for a config given as a dict."""
    rootfs = cfg.get("rootfs") or {}
    doc = {"architecture": cfg.get("architecture", "")}
    for k in ("author", "container"):
        if not _empty(cfg.get(k)):
            doc[k] = cfg[k]
    doc["created"] = cfg.get("created") or _ZERO_TIME
    if not _empty(cfg.get("docker_version")):
        doc["docker_version"] = cfg["docker_version"]
    if not _empty(cfg.get("history")):
        doc["history"] = [_go_history(h) for h in cfg["history"]]
    doc["os"] = cfg.get("os", "")
    doc["rootfs"] = {"type": rootfs.get("type", ""), "diff_ids": rootfs.get("diff_ids")}
    doc["config"] = _go_config(cfg.get("config") or {})
    for k in ("os.version", "variant", "os.features"):
        if not _empty(cfg.get(k)):
            doc[k] = cfg[k]
    lines: list = []
    _render(doc, "  ", lines, "", "")
    return "\n".join(lines).encode()


class ImageConfigSecretAnalyzer:
    """newSecretAnalyzer / Analyze (imgconf/secret/secret.go:26-62)."""

    def __init__(self, config_path: str = "", device: Optional[int] = None):
        try:
            cfg = S.parse_config(config_path)
        except S.ConfigError as e:
            raise S.ConfigError(f"secret config error: {e}") from e
        self.scanner = S.new_scanner(cfg, device)

    def required(self, _os=None) -> bool:
        return True

    def analyze(self, config: Optional[dict]) -> Optional[Secret]:
        if config is None:
            return None
        res = self.scanner.scan(S.ScanArgs("config.json", marshal_config_file(config)))
        return res if res.Findings else None
