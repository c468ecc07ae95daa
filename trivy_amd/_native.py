"""ctypes binding of the C ABI in include/trivy_secret_gpu.h.

The product path has exactly one implementation: libtrivy_secret_gpu.so (HIP
kernels for gfx950 + host C++).  If the library is missing this module raises
on import; if no GPU is visible, engine creation raises — there is no CPU
fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# TSG_LIB_VARIANT selects a diagnostic build of the same sources: "exp" = the
# ablation build (`make exp`, tools/*.sh only), "asan" = host ASan/UBSan
# (`make -f tools/asan.mk`, tests/test_asan.py on the CPU only), "alt" = the
# product build of another revision (tools/build_alt.sh: same-box A/B runs)
_VARIANT = os.environ.get("TSG_LIB_VARIANT", "")
LIB_PATH = os.path.join(
    _HERE, f"libtrivy_secret_gpu_{_VARIANT}.so" if _VARIANT in ("exp", "asan") or _VARIANT.startswith("alt") else "libtrivy_secret_gpu.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()); "
        "the secret engine has no CPU fallback")

lib = ctypes.CDLL(LIB_PATH)

TSG_OK = 0
TSG_ERR_INVALID_ARG = 1
TSG_ERR_REGEX = 2
TSG_ERR_DEVICE = 3
TSG_ERR_NO_DEVICE = 4
TSG_ERR_UNSUPPORTED = 5
TSG_ERR_INTERNAL = 6
TSG_ERR_PANIC = 7
TSG_ERR_FULL = 8

TSG_FILE_PATH_ALLOWED = 1
TSG_FILE_SPECIAL = 2
TSG_FILE_BINARY = 4

c_char_pp = ctypes.POINTER(ctypes.c_char_p)


class AllowRuleC(ctypes.Structure):
    _fields_ = [("id", ctypes.c_char_p), ("regex", ctypes.c_char_p), ("path", ctypes.c_char_p)]


class RuleC(ctypes.Structure):
    _fields_ = [
        ("id", ctypes.c_char_p),
        ("regex", ctypes.c_char_p),
        ("keywords", c_char_pp),
        ("n_keywords", ctypes.c_size_t),
        ("path", ctypes.c_char_p),
        ("secret_group_name", ctypes.c_char_p),
        ("allow_rules", ctypes.POINTER(AllowRuleC)),
        ("n_allow_rules", ctypes.c_size_t),
        ("exclude_regexes", c_char_pp),
        ("n_exclude_regexes", ctypes.c_size_t),
    ]


class FileC(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_uint64), ("path", ctypes.c_char_p)]


class LocC(ctypes.Structure):
    _fields_ = [("file", ctypes.c_uint32), ("rule", ctypes.c_uint32), ("start", ctypes.c_uint64),
                ("end", ctypes.c_uint64), ("start_line", ctypes.c_uint32), ("end_line", ctypes.c_uint32)]


class LineC(ctypes.Structure):
    _fields_ = [("number", ctypes.c_uint32), ("content", ctypes.c_void_p), ("content_len", ctypes.c_size_t),
                ("is_cause", ctypes.c_uint8), ("first_cause", ctypes.c_uint8), ("last_cause", ctypes.c_uint8)]


class FindingC(ctypes.Structure):
    _fields_ = [("file", ctypes.c_uint32), ("rule", ctypes.c_uint32), ("start_line", ctypes.c_uint32),
                ("end_line", ctypes.c_uint32), ("match", ctypes.c_void_p), ("match_len", ctypes.c_size_t),
                ("lines", ctypes.POINTER(LineC)), ("n_lines", ctypes.c_size_t),
                ("start", ctypes.c_uint64), ("end", ctypes.c_uint64)]


class TarEntryC(ctypes.Structure):
    _fields_ = [("path", ctypes.c_void_p), ("path_len", ctypes.c_size_t), ("offset", ctypes.c_uint64),
                ("size", ctypes.c_uint64), ("mode", ctypes.c_uint32), ("is_dir", ctypes.c_uint8)]


_SIGS = {
    "tsg_version": (ctypes.c_char_p, []),
    "tsg_last_error": (ctypes.c_char_p, []),
    "tsg_ruleset_compile": (ctypes.c_int, [ctypes.POINTER(RuleC), ctypes.c_size_t, ctypes.POINTER(AllowRuleC),
                                           ctypes.c_size_t, c_char_pp, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_size_t]),
    "tsg_ruleset_free": (None, [ctypes.c_void_p]),
    "tsg_ruleset_rule_count": (ctypes.c_size_t, [ctypes.c_void_p]),
    "tsg_ruleset_rule_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                             ctypes.POINTER(ctypes.c_size_t)]),
    "tsg_ruleset_rule_literal": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_char_p,
                                                ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "tsg_ruleset_scan_pattern": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                                ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint32),
                                                ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]),
    "tsg_ruleset_kw_states": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                             ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_size_t]),
    "tsg_ruleset_scan_image": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                              ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint32)]),
    "tsg_ruleset_rule_prog": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32),
                                             ctypes.POINTER(ctypes.c_uint32)]),
    "tsg_ruleset_group_span": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t] + [ctypes.POINTER(ctypes.c_int)] * 4),
    "tsg_ruleset_path_dfa_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p,
                                                  ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]),
    "tsg_ruleset_big_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.POINTER(ctypes.c_uint32)]),
    "tsg_ruleset_dfa_accel_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                                   ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint64)]),
    "tsg_ruleset_ac_visits": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_uint32)]),
    "tsg_engine_force_verify_split": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "tsg_diag_sort_pairs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "tsg_big_cold_lds_floor": (ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
    "tsg_ruleset_big_forge_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "tsg_ruleset_group_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint32),
                                             ctypes.POINTER(ctypes.c_uint32)]),
    "tsg_ruleset_dfa_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                             ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint32)]),
    "tsg_ruleset_nfa_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                             ctypes.c_size_t, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint32)]),
    "tsg_ruleset_follow_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                                ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                                ctypes.POINTER(ctypes.c_uint32)]),
    "tsg_ruleset_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int)]),
    "tsg_engine_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_engine_free": (None, [ctypes.c_void_p]),
    "tsg_scan": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(FileC), ctypes.c_size_t,
                                ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_scan_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_part_halo": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "tsg_scan_part_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                            ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p),
                                            ctypes.POINTER(ctypes.c_size_t)]),
    "tsg_part_free": (None, [ctypes.c_void_p]),
    "tsg_scan_merge_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p),
                                             ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_result_loc_count": (ctypes.c_size_t, [ctypes.c_void_p]),
    "tsg_result_locs": (ctypes.POINTER(LocC), [ctypes.c_void_p]),
    "tsg_result_file_count": (ctypes.c_size_t, [ctypes.c_void_p]),
    "tsg_result_file_flags": (ctypes.POINTER(ctypes.c_uint8), [ctypes.c_void_p]),
    "tsg_result_findings": (ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_size_t,
                                              ctypes.POINTER(ctypes.POINTER(FindingC))]),
    "tsg_result_timings": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_size_t)]),
    "tsg_result_free": (None, [ctypes.c_void_p]),
    "tsg_analyze": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(FileC), ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_staging_create": (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_staging_add": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_staging_count": (ctypes.c_size_t, [ctypes.c_void_p]),
    "tsg_staging_bytes": (ctypes.c_size_t, [ctypes.c_void_p]),
    "tsg_staging_reset": (None, [ctypes.c_void_p]),
    "tsg_staging_free": (None, [ctypes.c_void_p]),
    "tsg_analyze_staged": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_scan_staged": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_engine_gate_timings": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_size_t,
                                               ctypes.POINTER(ctypes.c_size_t)]),
    "tsg_gate_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t]),
    "tsg_regex_match": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_int)]),
    "tsg_regex_find_all": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_int64), ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_size_t)]),
    "tsg_layer_tar_walk": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, c_char_pp, ctypes.c_size_t,
                                          c_char_pp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_tar_walk_entry_count": (ctypes.c_size_t, [ctypes.c_void_p]),
    "tsg_tar_walk_entries": (ctypes.POINTER(TarEntryC), [ctypes.c_void_p]),
    "tsg_tar_walk_opq_count": (ctypes.c_size_t, [ctypes.c_void_p]),
    "tsg_tar_walk_opq_dir": (ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_size_t]),
    "tsg_tar_walk_wh_count": (ctypes.c_size_t, [ctypes.c_void_p]),
    "tsg_tar_walk_wh_file": (ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_size_t]),
    "tsg_tar_walk_free": (None, [ctypes.c_void_p]),
    "tsg_analyze_layer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_void_p)]),
    "tsg_ruleset_allow_path": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t,
                                              ctypes.POINTER(ctypes.c_int)]),
    "tsg_glob_match": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
}

for _name, (_res, _args) in _SIGS.items():
    if _VARIANT.startswith("alt") and not hasattr(lib, _name):
        continue  # (an older revision's build for A/B: diagnostics it predates stay unbound)
    _fn = getattr(lib, _name)  # AttributeError here = symbol missing from the .so
    _fn.restype = _res
    _fn.argtypes = _args

EXPORTED = sorted(_SIGS)

# The synthetic-corpus generator (bench.py, tests) lives in its own library,
# bench_gen/libtsg_corpus.so (header bench_gen/tsg_corpus.h), outside the
# product ABI; `gen` loads it on first use.
GEN_PATH = os.path.join(os.path.dirname(_HERE), "bench_gen", "libtsg_corpus.so")
_GEN_SIGS = {
    "tsg_gen_corpus_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_double, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "tsg_gen_file": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double,
                                    ctypes.c_void_p]),
    "tsg_gen_file_plants": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_size_t)]),
    "tsg_gen_file_nonascii": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32]),
    "tsg_gen_template_count": (ctypes.c_size_t, []),
    "tsg_gen_template_rule": (ctypes.c_char_p, [ctypes.c_size_t]),
    "tsg_gen_plant_record_size": (ctypes.c_size_t, []),
    "tsg_gen_chunk_bytes": (ctypes.c_uint32, []),
}


def __getattr__(name):
    if name != "gen":
        raise AttributeError(name)
    if not os.path.exists(GEN_PATH):
        raise ImportError(f"{GEN_PATH} is missing: build it with `make`")
    g = ctypes.CDLL(GEN_PATH)
    for fn_name, (res, args) in _GEN_SIGS.items():
        f = getattr(g, fn_name)
        f.restype = res
        f.argtypes = args
    globals()["gen"] = g
    return g


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[tsg {code}] {msg}")
        self.code = code


def check(rc):
    if rc != TSG_OK:
        raise EngineError(rc, lib.tsg_last_error().decode("utf-8", "replace"))


def regex_find_all(pattern: str, text: bytes, cap: int = 1 << 16):
    """Host compiler + VM diagnostics (FindAllIndex); not used by the scan path."""
    arr = (ctypes.c_int64 * (2 * cap))()
    n = ctypes.c_size_t()
    check(lib.tsg_regex_find_all(pattern.encode(), text, len(text), arr, cap, ctypes.byref(n)))
    return [[arr[2 * i], arr[2 * i + 1]] for i in range(min(n.value, cap))]


def regex_match(pattern: str, text: bytes) -> bool:
    m = ctypes.c_int()
    check(lib.tsg_regex_match(pattern.encode(), text, len(text), ctypes.byref(m)))
    return bool(m.value)


class DeviceBuffer:
    """A copy of a host numpy array in device memory, through the HIP runtime
    libtrivy_secret_gpu.so links (libamdhip64.so.7, already mapped), for the
    device-resident entry points (tsg_scan_device).  Test / tooling helper."""
    _hip = None

    def __init__(self, arr):
        if DeviceBuffer._hip is None:
            h = ctypes.CDLL("libamdhip64.so.7")
            h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
            h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            h.hipFree.argtypes = [ctypes.c_void_p]
            DeviceBuffer._hip = h
        self.ptr = ctypes.c_void_p()
        n = max(1, arr.nbytes)
        if DeviceBuffer._hip.hipMalloc(ctypes.byref(self.ptr), n) != 0:
            raise EngineError(TSG_ERR_DEVICE, "hipMalloc failed")
        if arr.nbytes and DeviceBuffer._hip.hipMemcpy(self.ptr, arr.ctypes.data, arr.nbytes, 1) != 0:  # H2D
            self.free()
            raise EngineError(TSG_ERR_DEVICE, "hipMemcpy failed")

    def free(self):
        if self.ptr:
            DeviceBuffer._hip.hipFree(self.ptr)
            self.ptr = ctypes.c_void_p()
