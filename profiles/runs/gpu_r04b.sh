#!/bin/bash
# r04b: per-wave k_report; GPU suite, configs[2] line + kernel timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r04b.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r04b.log; exit 1; }
tail -2 gpurun_out/pytest_r04b.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_c2_r04b.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r04b.log; exit 1; }
tail -1 gpurun_out/bench_c2_r04b.log | cut -c1-900
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c2b -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c2b.log 2>&1 || { echo "c2 trace failed"; tail -20 gpurun_out/c2b.log; exit 1; }
python3 tools/timeline.py gpurun_out/c2b/run_kernel_trace.csv k_scan_fast 12 > gpurun_out/c2b/timeline.txt
awk '$2>0.05 || $3>0.05' gpurun_out/c2b/timeline.txt
