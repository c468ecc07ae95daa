#!/bin/bash
# r04c: fast/slow k_verify split; GPU suite, configs[2] and configs[4] lines, c4 trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r04c.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r04c.log; exit 1; }
tail -2 gpurun_out/pytest_r04c.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_c2_r04c.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r04c.log; exit 1; }
tail -1 gpurun_out/bench_c2_r04c.log | cut -c1-700
timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 > gpurun_out/bench_c4_r04c.log 2>&1 || { echo "bench c4 failed"; tail -20 gpurun_out/bench_c4_r04c.log; exit 1; }
tail -1 gpurun_out/bench_c4_r04c.log | cut -c1-1500
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c4c -o run -- python3 -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu --no-parity > gpurun_out/c4c.log 2>&1 || { echo "c4 trace failed"; tail -20 gpurun_out/c4c.log; exit 1; }
python3 tools/timeline.py gpurun_out/c4c/run_kernel_trace.csv k_scan_big 12 > gpurun_out/c4c/timeline.txt
awk '$2>0.1 || $3>0.1' gpurun_out/c4c/timeline.txt
