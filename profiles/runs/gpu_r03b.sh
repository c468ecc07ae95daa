#!/bin/bash
# r03b: new device exclude path + shared-list bench tests, configs[4] 10 GB
# rocprof + verify profile, configs[2] kernel timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_exclude.py tests/test_bench_shared.py tests/test_gpu_parity.py > gpurun_out/pytest_r03b.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_r03b.log; exit 1; }
tail -2 gpurun_out/pytest_r03b.log
bash tools/c4_verify_prof.sh 10 c4r03b || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c2tl -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c2tl.log 2>&1 || { echo "c2 trace failed"; tail -20 gpurun_out/c2tl.log; exit 1; }
tail -1 gpurun_out/c2tl.log
python3 tools/timeline.py gpurun_out/c2tl/run_kernel_trace.csv k_scan_fast 12 > gpurun_out/c2tl/timeline.txt
python3 tools/timeline.py gpurun_out/c4r03b_prof/run_kernel_trace.csv k_scan_big 12 > gpurun_out/c4r03b_prof/timeline.txt
tail -3 gpurun_out/c2tl/timeline.txt
