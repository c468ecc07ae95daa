#!/usr/bin/env python3
"""Transcribe the reference's secret-scanner known-answer tests into JSON
fixtures under tests/golden/.

    python tools/extract_golden.py /root/reference

Sources (all read as text; nothing from the reference is executed):
  * pkg/fanal/secret/scanner_test.go:21-997          -> tests/golden/scanner_cases.json
  * pkg/fanal/secret/testdata/*                       -> tests/golden/secret_testdata/
  * pkg/fanal/analyzer/secret/secret_test.go:16-233   -> tests/golden/analyzer_cases.json
  * pkg/fanal/analyzer/secret/testdata/*              -> tests/golden/analyzer_testdata/
  * integration/testdata/secrets.json.golden + fixtures/repo/secrets/*
                                                      -> tests/golden/integration/
The input files and the expected structs are test *data* (inputs and expected
outputs); the Go test code itself is not copied.
"""
import json
import os
import re
import shutil
import sys

sys.path.insert(0, os.path.dirname(__file__))
from go_literal import Call, Composite, Ident, Parser  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "..", "tests", "golden")


CATEGORIES = {}


def load_categories(ref):
    src = open(os.path.join(ref, "pkg/fanal/secret/builtin-rules.go")).read()
    for m in re.finditer(r'(Category\w+)\s*=\s*types\.SecretRuleCategory\("([^"]*)"\)', src):
        CATEGORIES["secret." + m.group(1)] = m.group(2)


def ev(v, env):
    if isinstance(v, Ident):
        if v.name in CATEGORIES:
            return CATEGORIES[v.name]
        return env[v.name]
    if isinstance(v, Call):
        if v.name == "filepath.Join":
            return "/".join(ev(a, env) for a in v.args)
        raise ValueError(v.name)
    if isinstance(v, Composite):
        t = v.type or ""
        if t.startswith("[]"):
            return [ev(x, env) for x in v.items()]
        if t in ("types.SecretFinding",):
            return finding(v, env)
        # anonymous struct / types.Secret / analyzer.AnalysisResult
        if v.elems and all(k is None for k, _ in v.elems):
            return [ev(x, env) for x in v.items()]
        return {k: ev(x, env) for k, x in v.elems}
    return v


def line(v):
    f = v.fields()
    return {
        "Number": f.get("Number", 0),
        "Content": f.get("Content", ""),
        "IsCause": f.get("IsCause", False),
        "Annotation": f.get("Annotation", ""),
        "Truncated": f.get("Truncated", False),
        "Highlighted": f.get("Highlighted", ""),
        "FirstCause": f.get("FirstCause", False),
        "LastCause": f.get("LastCause", False),
    }


def finding(v, env):
    f = v.fields()
    code = f.get("Code")
    lines = []
    if code is not None:
        cl = code.fields().get("Lines")
        if cl is not None:
            lines = [line(x) for x in cl.items()]
    return {
        "RuleID": f.get("RuleID", ""),
        "Category": ev(f.get("Category", ""), env),
        "Severity": f.get("Severity", ""),
        "Title": f.get("Title", ""),
        "StartLine": f.get("StartLine", 0),
        "EndLine": f.get("EndLine", 0),
        "Code": {"Lines": lines},
        "Match": f.get("Match", ""),
    }


def parse_func(src, fname):
    """Parse `name := <literal>` statements and the tests table of a Go test
    function, returning (env, tests)."""
    start = src.index(f"func {fname}(")
    body = src[start:]
    stop = body.index("\n\tfor _, tt := range tests")
    body = body[body.index("{") + 1:stop]
    env = {}
    tests = None
    for m in re.finditer(r"\n\t(\w+) := ", body):
        name = m.group(1)
        p = Parser(body[m.end():])
        if name == "tests":
            # []struct{...}{ ... }: skip the struct type declaration
            p.take("[]")
            p.take()  # 'struct'
            depth = 0
            while True:
                _, v = p.take()
                if v == "{":
                    depth += 1
                elif v == "}":
                    depth -= 1
                    if depth == 0:
                        break
            lit = p.composite("[]case")
            tests = []
            for item in lit.items():
                tests.append({k: ev(x, env) for k, x in item.elems})
        else:
            env[name] = ev(p.value(), env)
    return env, tests


def copy_dir(src, dst):
    if os.path.exists(dst):
        shutil.rmtree(dst)
    shutil.copytree(src, dst)


def main(ref):
    os.makedirs(GOLD, exist_ok=True)
    load_categories(ref)
    # ---- pkg/fanal/secret ------------------------------------------------------
    sdir = os.path.join(ref, "pkg/fanal/secret")
    src = open(os.path.join(sdir, "scanner_test.go")).read()
    _, tests = parse_func(src, "TestSecretScanner")
    cases = []
    for t in tests:
        want = t["want"]
        cases.append({
            "name": t["name"],
            "config": t["configPath"].replace("testdata/", "secret_testdata/", 1),
            "input": t["inputFilePath"].replace("testdata/", "secret_testdata/", 1),
            "file_path": t["inputFilePath"],
            "want": {
                "FilePath": want.get("FilePath", ""),
                "Findings": want.get("Findings") or [],
            },
        })
    copy_dir(os.path.join(sdir, "testdata"), os.path.join(GOLD, "secret_testdata"))
    with open(os.path.join(GOLD, "scanner_cases.json"), "w") as fh:
        json.dump({"source": "pkg/fanal/secret/scanner_test.go:21-997", "cases": cases},
                  fh, indent=1, ensure_ascii=False)
    print(f"scanner cases: {len(cases)}")

    # ---- pkg/fanal/analyzer/secret ---------------------------------------------
    adir = os.path.join(ref, "pkg/fanal/analyzer/secret")
    asrc = open(os.path.join(adir, "secret_test.go")).read()
    _, atests = parse_func(asrc, "TestSecretAnalyzer")
    acases = []
    for t in atests:
        want = t.get("want")
        secrets = None
        if want:
            secrets = [{"FilePath": s.get("FilePath", ""), "Findings": s.get("Findings") or []}
                       for s in want["Secrets"]]
        acases.append({
            "name": t["name"],
            "config": t["configPath"].replace("testdata/", "analyzer_testdata/", 1),
            "file_path": t["filePath"],
            "input": t["filePath"].replace("testdata/", "analyzer_testdata/", 1),
            "dir": t.get("dir", ""),
            "want_secrets": secrets,
        })
    _, rtests = parse_func(asrc, "TestSecretRequire")
    rcases = [{"name": t["name"], "file_path": t["filePath"],
               "input": t["filePath"].replace("testdata/", "analyzer_testdata/", 1),
               "want": t["want"]} for t in rtests]
    copy_dir(os.path.join(adir, "testdata"), os.path.join(GOLD, "analyzer_testdata"))
    with open(os.path.join(GOLD, "analyzer_cases.json"), "w") as fh:
        json.dump({"source": "pkg/fanal/analyzer/secret/secret_test.go:16-233",
                   "analyze": acases, "required": rcases,
                   "required_config": "analyzer_testdata/skip-tests-config.yaml"},
                  fh, indent=1, ensure_ascii=False)
    print(f"analyzer cases: {len(acases)} analyze, {len(rcases)} required")

    # ---- integration golden ----------------------------------------------------
    idir = os.path.join(GOLD, "integration")
    copy_dir(os.path.join(ref, "integration/testdata/fixtures/repo/secrets"), os.path.join(idir, "repo"))
    shutil.copy(os.path.join(ref, "integration/testdata/secrets.json.golden"),
                os.path.join(idir, "secrets.json.golden"))
    print("integration golden copied")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
