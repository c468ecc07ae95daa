"""Pin the CPU oracle (oracle/secret_oracle.py) against the reference's own
known-answer tests, transcribed into tests/golden/ by tools/extract_golden.py.

pkg/fanal/secret/scanner_test.go:21-997, pkg/fanal/analyzer/secret/secret_test.go:16-233,
integration/testdata/secrets.json.golden.
"""
import dataclasses
import json
import os

import pytest

from oracle import secret_oracle as o

from .conftest import GOLDEN

_CASES = json.load(open(os.path.join(GOLDEN, "scanner_cases.json")))["cases"]
_ACASES = json.load(open(os.path.join(GOLDEN, "analyzer_cases.json")))


def _plain(secret):
    return {"FilePath": secret["FilePath"],
            "Findings": [{k: v for k, v in dataclasses.asdict(f).items() if k not in ("Start", "End")}
                         for f in secret["Findings"]]}


@pytest.mark.parametrize("case", _CASES, ids=[f"{i}-{c['name']}" for i, c in enumerate(_CASES)])
def test_scanner_case(case):
    content = open(os.path.join(GOLDEN, case["input"]), "rb").read().replace(b"\r", b"")
    sc = o.Scanner(o.parse_config(os.path.join(GOLDEN, case["config"])))
    assert _plain(sc.scan(case["file_path"], content)) == case["want"]


@pytest.mark.parametrize("case", _ACASES["analyze"], ids=[c["name"] for c in _ACASES["analyze"]])
def test_analyzer_case(case):
    cfg = os.path.join(GOLDEN, case["config"]) if case["config"] else ""
    a = o.SecretAnalyzer(cfg)
    content = open(os.path.join(GOLDEN, case["input"]), "rb").read()
    got = a.analyze(case["file_path"], content, case["dir"])
    if case["want_secrets"] is None:
        assert got is None
    else:
        assert [_plain(s) for s in got] == case["want_secrets"]


@pytest.mark.parametrize("case", _ACASES["required"], ids=[c["name"] for c in _ACASES["required"]])
def test_required_case(case):
    a = o.SecretAnalyzer(os.path.join(GOLDEN, _ACASES["required_config"]))
    size = os.path.getsize(os.path.join(GOLDEN, case["input"]))
    assert a.required(case["file_path"], size) == case["want"]


def test_integration_golden():
    """integration/repo_test.go:327-333: trivy repo --secret-config trivy-secret.yaml."""
    repo = os.path.join(GOLDEN, "integration", "repo")
    golden = json.load(open(os.path.join(GOLDEN, "integration", "secrets.json.golden")))
    want = [r for r in golden["Results"] if r.get("Class") == "secret"]
    a = o.SecretAnalyzer(os.path.join(repo, "trivy-secret.yaml"))
    got = []
    for name in sorted(os.listdir(repo)):
        data = open(os.path.join(repo, name), "rb").read()
        if not a.required(name, len(data)):
            continue
        res = a.analyze(name, data, ".")
        if res:
            got.extend(res)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g["FilePath"] == w["Target"]
        gf = sorted(_plain(g)["Findings"], key=lambda f: (f["RuleID"], f["StartLine"]))
        for f, wf in zip(gf, w["Secrets"]):
            for k in ("RuleID", "Category", "Severity", "Title", "StartLine", "EndLine", "Match"):
                assert f[k] == wf[k], k
            for gl, wl in zip(f["Code"]["Lines"], wf["Code"]["Lines"]):
                assert gl["Number"] == wl["Number"] and gl["Content"] == wl["Content"]
                assert gl["IsCause"] == wl["IsCause"]
