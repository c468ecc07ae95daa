#!/bin/bash
# r04e: verify split with k_allow + run acceleration: GPU suite, c2 line + timeline, c4 line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r04e.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r04e.log; exit 1; }
tail -2 gpurun_out/pytest_r04e.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_c2_r04e.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r04e.log; exit 1; }
tail -1 gpurun_out/bench_c2_r04e.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['counts'], d['parity']['spot_mismatched_files'], d['parity']['planted_found'], d['parity']['decoys_found'])"
timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c4_r04e.log 2>&1 || { echo "bench c4 failed"; tail -20 gpurun_out/bench_c4_r04e.log; exit 1; }
tail -1 gpurun_out/bench_c4_r04e.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['counts'], d['parity']['stress_mismatched_files'], d['parity']['spot_mismatched_files'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c2e -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c2e.log 2>&1 || { echo "c2 trace failed"; tail -20 gpurun_out/c2e.log; exit 1; }
python3 tools/timeline.py gpurun_out/c2e/run_kernel_trace.csv k_scan_fast 12 > gpurun_out/c2e/timeline.txt
awk '$2>0.05 || $3>0.03' gpurun_out/c2e/timeline.txt
