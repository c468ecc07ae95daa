"""Host-side ASan + UBSan run of the C ABI (sanitizers on host
code only — the GPU pool has no device ASan).

Re-runs the host-only tests — malformed-tar fuzz and threaded reentrancy
(test_robustness.py), the layer-tar walker vs the oracle (test_layertar.py),
the scan-automaton extension soundness (test_scan_ext.py) and the host-logic
checks — in a child process that loads trivy_amd/libtrivy_secret_gpu_asan.so
(`make -f tools/asan.mk`, built by __graft_entry__.build()) under the clang
ASan runtime.  Any sanitizer report aborts the child and fails this test.
CPU only."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_LIB = os.path.join(ROOT, "trivy_amd", "libtrivy_secret_gpu_asan.so")
RUNTIMES = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))

# the four slowest host checks (VM-vs-oracle sweeps, minutes under ASan) stay
# in the plain CPU run only
SLOW = ("follow_filter_never_drops_a_match", "rune_symbols_equal_vm", "equals_vm_on_builtin_rules",
        "host_vm_matches_oracle_on_builtin_rules")


@pytest.mark.skipif(not RUNTIMES, reason="clang ASan runtime not found under /opt/rocm/lib/llvm")
def test_host_abi_under_asan_ubsan():
    # incremental: a no-op when __graft_entry__.build() already made it
    mk = subprocess.run(["make", "-s", "-f", "tools/asan.mk", "-j", str(min(8, os.cpu_count() or 4))], cwd=ROOT,
                        capture_output=True, text=True, timeout=1200)
    assert mk.returncode == 0 and os.path.exists(ASAN_LIB), mk.stdout[-2000:] + mk.stderr[-2000:]
    env = dict(os.environ)
    env.update(
        LD_PRELOAD=RUNTIMES[-1],
        TSG_LIB_VARIANT="asan",
        ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
        UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
    )
    probe = subprocess.run([sys.executable, "-c", "import trivy_amd._native as N; print(N.LIB_PATH)"], cwd=ROOT,
                           env=env, capture_output=True, text=True, timeout=300)
    assert probe.returncode == 0 and probe.stdout.strip() == ASAN_LIB, probe.stdout + probe.stderr
    tests = ["tests/test_robustness.py", "tests/test_layertar.py", "tests/test_scan_ext.py",
             "tests/test_host_logic.py"]
    cmd = [sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
           "-k", " and ".join(f"not {s}" for s in SLOW), *tests]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert "runtime error:" not in out, out[-4000:]
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert " passed" in out
