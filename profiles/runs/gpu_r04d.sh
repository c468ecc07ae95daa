#!/bin/bash
# r04d: configs[2] with the verify split: line (deferred count) + kernel timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_c2_r04d.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r04d.log; exit 1; }
tail -1 gpurun_out/bench_c2_r04d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'], d['counts'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c2d -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c2d.log 2>&1 || { echo "c2 trace failed"; tail -20 gpurun_out/c2d.log; exit 1; }
python3 tools/timeline.py gpurun_out/c2d/run_kernel_trace.csv k_scan_fast 12 > gpurun_out/c2d/timeline.txt
awk 'NR>14' gpurun_out/c2d/timeline.txt | head -60
