#!/bin/bash
# r04a: empty-match GPU tests, full GPU suite, configs[2] line, PMC passes for configs[2] and configs[4]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_empty_match.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r04a_empty.log 2>&1 || { echo "empty-match tests failed"; tail -60 gpurun_out/pytest_r04a_empty.log; exit 1; }
tail -3 gpurun_out/pytest_r04a_empty.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r04a.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r04a.log; exit 1; }
tail -2 gpurun_out/pytest_r04a.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_c2_r04a.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r04a.log; exit 1; }
tail -1 gpurun_out/bench_c2_r04a.log | cut -c1-1200
bash tools/pmc.sh r04a_c2 2 && bash tools/pmc.sh r04a_c4 4
