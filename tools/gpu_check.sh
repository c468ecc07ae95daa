#!/bin/bash
# One GPU round trip: parity tests, smoke, then bench lines (one per config
# given, e.g. `bash tools/gpu_check.sh 4 2`; none = tests + smoke only).
# Usage (from the repo root, on the GPU box).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
for cfg in "$@"; do
  timeout -k 10 500 python -u bench.py --config "$cfg" --steps 5 --warmup 2 > gpurun_out/bench_c$cfg.log 2>&1 || { echo "bench c$cfg failed"; tail -20 gpurun_out/bench_c$cfg.log; exit 1; }
  tail -1 gpurun_out/bench_c$cfg.log
done
