#!/bin/bash
# r03h: GPU suite, configs[4] line + timeline, split bench 20 GB, configs[2] line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_r03h.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r03h.log; exit 1; }
tail -2 gpurun_out/pytest_r03h.log
timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 2 > gpurun_out/bench_c4_r03h.log 2>&1 || { echo "bench c4 failed"; tail -20 gpurun_out/bench_c4_r03h.log; exit 1; }
tail -1 gpurun_out/bench_c4_r03h.log | cut -c1-1200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c4h -o run -- python3 -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c4h.log 2>&1 || { echo "c4 trace failed"; tail -20 gpurun_out/c4h.log; exit 1; }
python3 tools/timeline.py gpurun_out/c4h/run_kernel_trace.csv k_scan_big 12 > gpurun_out/c4h/timeline.txt
awk '$2>0.05 || $3>0.05' gpurun_out/c4h/timeline.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_c2_r03h.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r03h.log; exit 1; }
tail -1 gpurun_out/bench_c2_r03h.log | cut -c1-700
