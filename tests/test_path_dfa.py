"""Path regexes through the MatchString DFA the path gate walks (ruleset.cpp
path_dfa: the DFA of (?s:.)*?(?:re), anchored at 0) against the oracle's
MatchString (Rule.MatchPath / AllowPath, pkg/fanal/secret/scanner.go:391,397):
the builtin rules' allow paths, the configs[4] stress family's path, and
hand-written path regexes with anchors, alternations and classes.  CPU only
(host ABI + oracle)."""
import ctypes
import random

import pytest

from oracle import secret_oracle as O

N = pytest.importorskip("trivy_amd._native")
S = pytest.importorskip("trivy_amd.secret")

PATHS = ["a.env", "x/y/z.cfg", "src/app/main.go", "node_modules/x/index.js", "test/fixtures/a.txt", ".env",
         "env", "dir.env/file", "a/b/c/d/e/f.txt", "vendor/github.com/x.go", "README.md", "", "a\nb.env",
         "docs/x.md", "k8s/secret.yaml", "some path with spaces.cfg", "ñandú/é.txt", "tests/unit/x_test.go"]


def _paths(seed, n):
    rng = random.Random(seed)
    parts = ["src", "test", "tests", "node_modules", "vendor", "docs", "a", ".git", "x.env", "cfg", "examples"]
    exts = ["env", "cfg", "txt", "js", "go", "md", "yaml", "ENV", "Cfg", "py", "lock", ""]
    out = list(PATHS)
    for _ in range(n):
        p = "/".join(rng.choice(parts) for _ in range(rng.randint(0, 4)))
        f = "f%d" % rng.randint(0, 99) + ("." + rng.choice(exts) if rng.random() < 0.9 else "")
        out.append((p + "/" + f) if p else f)
    return out


def _check(sc, want_rules):
    checked = 0
    for i, r in enumerate(sc.rules):
        for which, src in ((0, r.path), (1, (r.allow_rules[0].path if r.allow_rules and r.allow_rules[0].path
                                             else None))):
            if not src:
                continue
            rx = O.GoRegexp(src)
            for p in _paths(i + which, 300):
                res = ctypes.c_int()
                b = p.encode()
                N.check(N.lib.tsg_ruleset_path_dfa_check(sc._rs.handle, i, which, b, len(b), ctypes.byref(res)))
                if res.value == 2:
                    continue
                assert bool(res.value) == rx.match_string(b), (r.id, src, p)
                checked += 1
    assert checked >= want_rules * 100, checked


def test_custom_path_regexes_dfa_equals_matchstring():
    srcs = [r".*\.(?:env|cfg|txt)$", r"^src/", r"(?i)\.ENV$", r"node_modules|vendor", r"^[a-z]+/[^/]*\.go$",
            r"tests?/", r"\.md$", r"^$", r"(^|/)\.env$"]
    custom = [S.Rule(id=f"p{k}", regex="zzq[0-9]{4}", keywords=["zzq"], path=src,
                     allow_rules=[S.AllowRule(id=f"a{k}", path=srcs[(k + 3) % len(srcs)])])
              for k, src in enumerate(srcs)]
    sc = S.new_scanner(S.Config(enable_builtin_rule_ids=["__none__"], custom_rules=custom))
    _check(sc, len(srcs))


def test_builtin_global_allow_paths_dfa_equals_matchstring():
    """The builtin allow rules' paths (Global.AllowPath, scanner.go:375):
    node_modules, vendor, tests, .md and friends."""
    srcs = [a.path for a in S.BUILTIN_ALLOW_RULES if a.path]
    assert len(srcs) >= 5
    sc = S.new_scanner(None)
    checked = 0
    for k, src in enumerate(srcs):
        rx = O.GoRegexp(src)
        for p in _paths(100 + k, 400) + ["a/node_modules/b.js", "x/vendor/y.go", "README.md", "docs/a.md"]:
            res = ctypes.c_int()
            b = p.encode()
            N.check(N.lib.tsg_ruleset_path_dfa_check(sc._rs.handle, k, 2, b, len(b), ctypes.byref(res)))
            if res.value == 2:
                continue
            assert bool(res.value) == rx.match_string(b), (src, p)
            checked += 1
    assert checked >= 300 * len(srcs), checked


def test_host_allow_path_dfa_equals_vm():
    """tsg_ruleset_allow_path (SecretAnalyzer.Required's global AllowPath,
    scanner.go:200-207) now decides paths with the path DFAs and falls back
    to the Pike VM only where a DFA cannot: on random paths built from the
    builtin allow rules' vocabulary (ASCII, upper case, non-ASCII, invalid
    UTF-8) it must equal MatchString of every rule on the VM alone."""
    import ctypes
    import json
    import os
    import random

    import trivy_amd._native as N
    import trivy_amd.secret as S

    data = json.load(open(os.path.join(os.path.dirname(S.__file__), "data", "builtin_rules.json")))
    pats = [a["path"] for a in data["allow_rules"] if a.get("path")]
    sc = S.new_scanner(None)
    rng = random.Random(41)
    words = ["test", "tests", "_test", "-test", ".test", "vendor", "example", "Example", "node_modules", "docs",
             "README.md", "a.md", "usr", "share", "doc", "src", "main.go", "lib", "x.min.js", "é", "ſ", "K",
             "pkg", "testdata", "mock", "spec", ".git", "a" * 40]
    paths = []
    for _ in range(4000):
        p = "/".join(rng.choice(words) for _ in range(rng.randint(1, 6)))
        if rng.random() < 0.3:
            p = "/" + p
        paths.append(p.encode("utf-8"))
    paths += [b"\xff/vendor/x", b"test\xc3", b"a/\xe2\x80/test"]
    for p in paths:
        want = False
        for r in pats:
            m = ctypes.c_int()
            N.check(N.lib.tsg_regex_match(r.encode(), p, len(p), ctypes.byref(m)))
            want = want or bool(m.value)
        got = ctypes.c_int()
        N.check(N.lib.tsg_ruleset_allow_path(sc._rs.handle, p, len(p), ctypes.byref(got)))
        assert bool(got.value) == want, p
