"""CPU-only tests of the host side: the C-ABI library loads and exports every
symbol include/trivy_secret_gpu.h declares; the Go-RE2 compiler + Pike VM
(host build of the same code the GPU runs) agree with the oracle; the rule
compiler classifies builtin rules; config parsing mirrors ParseConfig."""
import json
import os
import re

import pytest

from oracle import secret_oracle as o

from . import corpus_gen
from .conftest import GOLDEN, ROOT

N = pytest.importorskip("trivy_amd._native")
import trivy_amd.secret as S  # noqa: E402


def _decls(name):
    return set(re.findall(r"\b(tsg_[a-z_]+)\s*\(", open(os.path.join(ROOT, "include", name)).read()))


def test_header_symbols_exported():
    """Every entry point of the drop-in ABI (trivy_secret_gpu.h) and of the
    diagnostic header (trivy_secret_gpu_diag.h) is exported; the two are
    disjoint, and the diagnostic hooks stay out of the drop-in header."""
    abi, diag = _decls("trivy_secret_gpu.h"), _decls("trivy_secret_gpu_diag.h")
    assert abi and diag and not abi & diag
    for name in abi | diag:
        assert hasattr(N.lib, name), name
    assert set(N.EXPORTED) <= abi | diag
    assert not any(n.endswith("_check") or n in ("tsg_ruleset_scan_image", "tsg_ruleset_scan_pattern",
                                                 "tsg_regex_find_all") for n in abi)


def test_staging_contract_without_gpu():
    """The caller-filled staging API (tsg_staging_*): NULL handles are
    rejected and, without a GPU, creating the page-locked buffer fails with
    TSG_ERR_DEVICE -- no CPU fallback, no crash (the GPU behaviour, including
    TSG_ERR_FULL and reset, is tests/test_gpu_staging.py)."""
    import ctypes

    import torch

    d = ctypes.c_void_p()
    assert N.lib.tsg_staging_add(None, b"x", 5, ctypes.byref(d)) == N.TSG_ERR_INVALID_ARG
    assert N.lib.tsg_staging_count(None) == 0 and N.lib.tsg_staging_bytes(None) == 0
    N.lib.tsg_staging_reset(None)
    N.lib.tsg_staging_free(None)
    r = ctypes.c_void_p()
    assert N.lib.tsg_analyze_staged(None, None, None, ctypes.byref(r)) == N.TSG_ERR_INVALID_ARG
    assert N.lib.tsg_scan_staged(None, None, None, ctypes.byref(r)) == N.TSG_ERR_INVALID_ARG
    h = ctypes.c_void_p()
    assert N.lib.tsg_staging_create(0, ctypes.byref(h)) == N.TSG_ERR_INVALID_ARG
    if not torch.cuda.is_available():
        assert N.lib.tsg_staging_create(1 << 20, ctypes.byref(h)) == N.TSG_ERR_DEVICE and not h.value


def test_version():
    assert b"gfx950" in N.lib.tsg_version()


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    sc = S.new_scanner(None)
    with pytest.raises(N.EngineError):
        sc.scan(S.ScanArgs("a.txt", b"ghp_" + b"a" * 36))


_BUILTIN = json.load(open(os.path.join(ROOT, "trivy_amd", "data", "builtin_rules.json")))


def test_host_vm_matches_oracle_on_builtin_rules():
    files = corpus_gen.make_corpus(99, 120)
    files += [(c, open(os.path.join(GOLDEN, "secret_testdata", c), "rb").read())
              for c in os.listdir(os.path.join(GOLDEN, "secret_testdata")) if not c.endswith(".yaml")]
    n = 0
    for r in _BUILTIN["rules"]:
        g = o.GoRegexp(r["regex"])
        for _, data in files:
            want = g.find_all_index(data)
            n += len(want)
            assert N.regex_find_all(r["regex"], data) == want, (r["id"], data[:80])
    assert n > 100


@pytest.mark.parametrize("pat,text", [
    (r"a*", b"baaac"), (r"(?m)^x$", b"x\nx\n"), (r"^x$", b"x\nx"), (r"\bfoo\b", b"foo foobar foo"),
    (r"(a|ab)(c|bcd)(d*)", b"abcd"), (r"x*?y", b"xxy"), (r"(?i)k", "KKk".encode()),
    (r"(?i)s+", "sSſ".encode()), (r".", b"\xff\xc3\xa9\xe2\x82"), (r"[^a]", b"\xffa\n"),
    (r"(?U)a+", b"aaa"), (r"a{2,3}", b"aaaaaaa"), (r"(|a)*", b"aa"), (r"(a*)*", b"b"),
    (r"\Qa.b\E+", b"a.bbb a.b"), (r"[[:alpha:]]+", b"ab1cd"), (r"\x41\x{42}", b"AB"), (r"a|", b"xa"),
    (r"(?s).+", b"a\nb"), (r"$", b"ab\n"), (r"(?m)$", b"a\nb"), (r"\B", b"ab"),
])
def test_host_vm_semantics(pat, text):
    assert N.regex_find_all(pat, text) == o.GoRegexp(pat).find_all_index(text)


@pytest.mark.parametrize("bad", ["a**", "(", "[a", "a{2,1}", "x{1001}", "\\1", "(?P<>a)", "[z-a]", "*a"])
def test_regex_syntax_errors(bad):
    with pytest.raises(N.EngineError):
        N.regex_find_all(bad, b"")


def test_builtin_rules_compile_and_are_anchored():
    sc = S.new_scanner(None)
    import ctypes
    modes = []
    for i in range(len(sc.rules)):
        m = ctypes.c_int()
        a = ctypes.c_uint32()
        b = ctypes.c_uint32()
        k = ctypes.c_size_t()
        N.check(N.lib.tsg_ruleset_rule_info(sc._rs.handle, i, ctypes.byref(m), ctypes.byref(a),
                                            ctypes.byref(b), ctypes.byref(k)))
        modes.append(m.value)
    # every builtin rule gets a literal anchor (mode 1), none needs a full-file scan
    assert modes == [1] * len(sc.rules)


def test_parse_config_mirrors_reference():
    cfg = S.parse_config(os.path.join(GOLDEN, "secret_testdata", "config-with-non-uppercase-severity.yaml"))
    assert cfg.custom_rules[0].severity == "UNKNOWN"  # "uNknown" upper-cased (scanner.go:305-313)
    assert S.convert_severity("hIgh") == "HIGH" and S.convert_severity("bogus") == "UNKNOWN"
    assert S.parse_config("") is None
    assert S.parse_config("/nonexistent/trivy-secret.yaml") is None
    bad = os.path.join(GOLDEN, "..", "tmp_bad.yaml")
    try:
        with open(bad, "w") as fh:
            fh.write("rules:\n  - id: x\n    regex: 'a**'\n")
        with pytest.raises(S.ConfigError):
            S.parse_config(bad)
    finally:
        os.remove(bad)


def test_new_scanner_filters():
    cfg = S.parse_config(os.path.join(GOLDEN, "secret_testdata", "config-enable-ghp.yaml"))
    sc = S.new_scanner(cfg)
    assert [r.id for r in sc.rules] == [r.id for r in o.Scanner(o.parse_config(
        os.path.join(GOLDEN, "secret_testdata", "config-enable-ghp.yaml"))).rules]


def test_allow_path_host():
    sc = S.new_scanner(None)
    assert sc.allow_path("foo/README.md")
    assert sc.allow_path("/usr/share/doc/x") is False  # '^usr/' does not match a '/'-prefixed path
    assert sc.allow_path("usr/share/doc/x")
    assert not sc.allow_path("src/main.go")
