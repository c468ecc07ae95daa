"""Trivy's JSON report for secret findings (host side of the drop-in path).

Restates what a Trivy user reads after a secret scan:
  * pkg/scanner/local/scan.go:263-281 `secretsToResults`: one Result per
    Secret, Target = FilePath, Class "secret", Secrets = its findings as-is;
  * pkg/types/report.go:13-19,104-120 and pkg/fanal/types/secret.go:10-20,
    misconf.go:53-62: field order and omitempty (`Highlighted` omitted when
    empty; `Layer` rendered as `{}` -- a struct is never empty for omitempty);
  * pkg/report/json.go:20-30: json.MarshalIndent(report, "", "  ") plus a
    newline, with encoding/json's string escaping (HTML characters and
    U+2028/U+2029 as \\u escapes; each byte of invalid UTF-8 -- a rune
    utf8.DecodeRuneInString returns as RuneError of width 1 -- as the
    six-character escape \\ufffd, while a valid U+FFFD stays raw).

The findings come from the engine (device-built Match / Code), so this module
only formats; it never scans.

Contract for invalid UTF-8: strings in findings carry each byte Go's decoder
rejects as a lone surrogate (U+DC80-U+DCFF, Python's `surrogateescape`), and
the dicts `line_json` / `finding_json` / `secret_results` return keep them so,
because one dict string cannot tell Go's `\ufffd` escape text (an invalid
byte) from a raw U+FFFD (a valid rune).  Only `dumps()` / `report_json()`
produce Go's bytes; other serialisers of those dicts must either pass them
through `dumps()` or encode with `surrogateescape` (which gives back the raw
bytes, not Go's escapes).
"""
from __future__ import annotations

import json
import re
from typing import Iterable, List, Optional

from .types import Secret

_GO_ESCAPES = {"<": "\\u003c", ">": "\\u003e", "&": "\\u0026", " ": "\\u2028", " ": "\\u2029"}


# surrogateescape'd bytes (U+DC80-U+DCFF) are exactly the bytes Go's decoder
# rejects one at a time; dumps() writes each as the escape text \ufffd
_INVALID = re.compile("[\udc80-\udcff]")


def line_json(ln) -> dict:
    d = {"Number": ln.Number, "Content": ln.Content, "IsCause": ln.IsCause,
         "Annotation": ln.Annotation, "Truncated": ln.Truncated}
    if ln.Highlighted:
        d["Highlighted"] = ln.Highlighted
    d["FirstCause"] = ln.FirstCause
    d["LastCause"] = ln.LastCause
    return d


def finding_json(f) -> dict:
    return {"RuleID": f.RuleID, "Category": f.Category, "Severity": f.Severity, "Title": f.Title,
            "StartLine": f.StartLine, "EndLine": f.EndLine,
            "Code": {"Lines": [line_json(ln) for ln in f.Code.Lines] if f.Code.Lines else None},
            "Match": f.Match, "Layer": {}}


def secret_results(secrets: Iterable[Optional[Secret]]) -> List[dict]:
    """secretsToResults (scan.go:263-281); files without findings give none."""
    out = []
    for s in secrets:
        if s is None or not s.Findings:
            continue
        out.append({"Target": s.FilePath, "Class": "secret", "Secrets": [finding_json(f) for f in s.Findings]})
    return out


def dumps(obj) -> str:
    """json.MarshalIndent(obj, "", "  ") + "\\n" (json.go:21-27)."""
    text = json.dumps(obj, indent=2, ensure_ascii=False, separators=(",", ": "))
    for k, v in _GO_ESCAPES.items():
        text = text.replace(k, v)
    return _INVALID.sub(lambda m: "\\ufffd", text) + "\n"


def report_json(secrets: Iterable[Optional[Secret]], artifact_name: str = "", artifact_type: str = "",
                created_at: str = "", metadata: Optional[dict] = None, schema_version: int = 2) -> str:
    """A types.Report holding the secret Results, omitempty as report.go:13-19."""
    rep = {}
    if schema_version:
        rep["SchemaVersion"] = schema_version
    if created_at:
        rep["CreatedAt"] = created_at
    if artifact_name:
        rep["ArtifactName"] = artifact_name
    if artifact_type:
        rep["ArtifactType"] = artifact_type
    rep["Metadata"] = metadata if metadata is not None else {"ImageConfig": {
        "architecture": "", "created": "0001-01-01T00:00:00Z", "os": "",
        "rootfs": {"type": "", "diff_ids": None}, "config": {}}}
    results = secret_results(secrets)
    if results:
        rep["Results"] = results
    return dumps(rep)
