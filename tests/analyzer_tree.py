"""Test helpers for the AnalyzerGroup mirror (trivy_amd.analyzer): a source
tree whose secrets sit also in files other analyzers claim, the claiming
analyzers, and the reference's expected secrets -- SecretAnalyzer.Analyze per
required file (pkg/fanal/analyzer/secret/secret.go:79-153, restated by the
oracle) merged and sorted as AnalysisResult.Sort does (analyzer.go:218-229)."""
from __future__ import annotations

import dataclasses
import json
import os
import random

from oracle import secret_oracle as o
from trivy_amd.analyzer import AnalysisResult, Application, walk_local
from trivy_amd.types import Code, Line, Secret, SecretFinding

from . import corpus_gen

GHP = "ghp_" + "R" * 36


def make_tree(root: str, seed: int, n: int = 120) -> None:
    """corpus files plus: requirements.txt (claimed by pip) and
    usr/bin/tool.sh (listed by the dpkg analyzer's SystemInstalledFiles), both
    holding secrets; a binary; a CRLF file; skipped dirs / files / exts; a
    file under 10 bytes."""
    rng = random.Random(seed)
    files = corpus_gen.make_corpus(seed, n)
    extra = [
        ("requirements.txt", f"requests==2.31.0\n# token: {GHP}\nflask==3.0\n".encode()),
        ("sub/requirements.txt", b"numpy==2.2\n" + f"AWS_ACCESS_KEY_ID=AKIA{'B' * 16}\n".encode()),
        ("var/lib/dpkg/status", b"Package: tool\nStatus: install ok installed\n"),
        ("usr/bin/tool.sh", f"#!/bin/sh\nexport GITHUB_TOKEN={GHP}\n".encode()),
        ("bin/blob.dat", b"\x00\x01\x02" + GHP.encode()),
        ("win/crlf.env", f"a=1\r\ntoken: {GHP}\r\n".encode()),
        (".git/config", f"token = {GHP}\n".encode()),
        ("node_modules/x/index.js", f"const t = '{GHP}'\n".encode()),
        ("go.sum", f"{GHP}\n".encode()),
        ("img/logo.png", f"{GHP}\n".encode()),
        ("tiny.txt", b"short"),
    ]
    for p, d in files + extra:
        if rng.random() < 0.1:
            d = d.replace(b"\n", b"\r\n")
        f = os.path.join(root, p)
        os.makedirs(os.path.dirname(f), exist_ok=True)
        with open(f, "wb") as fh:
            fh.write(d)


class PipAnalyzer:
    """A language analyzer that claims requirements.txt (types.Application)."""

    def type(self):
        return "pip"

    def version(self):
        return 1

    def required(self, path, info):
        return os.path.basename(path) == "requirements.txt"

    def analyze_input(self, inp):
        return AnalysisResult(applications=[Application("pip", inp.file_path)])


class DpkgAnalyzer:
    """An OS-package analyzer whose result lists installed files."""

    def type(self):
        return "dpkg"

    def version(self):
        return 1

    def required(self, path, info):
        return path == "var/lib/dpkg/status"

    def analyze_input(self, inp):
        return AnalysisResult(system_installed_files=["usr/bin/tool.sh"])


class RecordingPostAnalyzer:
    """A post-analyzer of another type that requires every file and records
    the (filtered) FS it is handed."""

    def __init__(self):
        self.seen = None
        self.inits = 0

    def init(self, opts):
        self.inits += 1
        return self

    def type(self):
        return "jar"

    def version(self):
        return 1

    def required(self, path, info):
        return True

    def post_analyze(self, fsys):
        self.seen = set(fsys.files)
        return None


def to_secret(r) -> Secret:
    """An oracle result dict -> types.Secret."""
    fs = []
    for f in r["Findings"]:
        d = {k: v for k, v in dataclasses.asdict(f).items() if k not in ("Start", "End")}
        d["Code"] = Code(Lines=[Line(**ln) for ln in d["Code"]["Lines"]])
        fs.append(SecretFinding(**d))
    return Secret(FilePath=r["FilePath"], Findings=fs)


def oracle_go_analyze(config_path: str = ""):
    """Trivy's per-file SecretAnalyzer.Analyze (the pure-Go Scanner of the
    tagged build's fallback), restated by the oracle."""
    oa = o.SecretAnalyzer(config_path)

    def go_analyze(path, raw, dir_):
        r = oa.analyze(path, raw, dir_)
        return [to_secret(x) for x in r] if r else None
    return go_analyze


def reference_secrets(root: str, config_path: str = ""):
    """The reference: Analyze of every file SecretAnalyzer.Required accepts
    (Dir = the root: no '/' prefix), claimed files included, sorted."""
    oa = o.SecretAnalyzer(config_path)
    out = []
    for rel, info in walk_local(root):
        if not oa.required(rel, info.size):
            continue
        with open(info.real, "rb") as f:
            r = oa.analyze(rel, f.read(), root)
        if r:
            out += [to_secret(x) for x in r]
    res = AnalysisResult(secrets=out)
    res.sort()
    return res.secrets


def canon(secrets):
    """Secrets as comparable JSON (order as given: AnalysisResult.Sort has
    already ordered them; findings of equal (RuleID, StartLine) compared as
    sets)."""
    out = []
    for s in secrets:
        fs = [json.dumps(dataclasses.asdict(f), sort_keys=True) for f in s.Findings]
        out.append((s.FilePath, sorted(fs)))
    return out
