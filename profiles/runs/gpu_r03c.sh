#!/bin/bash
# r03c: 64-bit match-search instantiations (files past 2^31 / 2^32): full GPU
# suite, smoke, configs[2] and configs[4] lines, split bench on a 5 GB file.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_r03c.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r03c.log; exit 1; }
tail -2 gpurun_out/pytest_r03c.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_c2_r03c.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r03c.log; exit 1; }
tail -1 gpurun_out/bench_c2_r03c.log | cut -c1-900
timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 2 > gpurun_out/bench_c4_r03c.log 2>&1 || { echo "bench c4 failed"; tail -20 gpurun_out/bench_c4_r03c.log; exit 1; }
tail -1 gpurun_out/bench_c4_r03c.log | cut -c1-1500
timeout -k 10 300 python -u tools/split_bench.py --gb 5 --parts 2 4 8 > gpurun_out/split_bench_r03c.log 2>&1 || { echo "split bench failed"; tail -20 gpurun_out/split_bench_r03c.log; exit 1; }
tail -1 gpurun_out/split_bench_r03c.log
