#!/bin/bash
# r03k: GPU suite, configs[4] line + timeline (k_big_walk / k_big_resolve,
# 8-byte cold records), configs[2] line, then the k_scan_big A/B (exp build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_r03k.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r03k.log; exit 1; }
tail -2 gpurun_out/pytest_r03k.log
timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 2 > gpurun_out/bench_c4_r03k.log 2>&1 || { echo "bench c4 failed"; tail -20 gpurun_out/bench_c4_r03k.log; exit 1; }
tail -1 gpurun_out/bench_c4_r03k.log | cut -c1-1500
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c4k -o run -- python3 -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c4k.log 2>&1 || { echo "c4 trace failed"; tail -20 gpurun_out/c4k.log; exit 1; }
python3 tools/timeline.py gpurun_out/c4k/run_kernel_trace.csv k_scan_big 12 > gpurun_out/c4k/timeline.txt
awk '$2>0.05 || $3>0.05' gpurun_out/c4k/timeline.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_c2_r03k.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r03k.log; exit 1; }
tail -1 gpurun_out/bench_c2_r03k.log | cut -c1-700
export TSG_LIB_VARIANT=exp
for v in 0 1 2 4 0x2v2 8x2v2 12x2v2; do
  export TSG_BIG_VARIANT=$v
  timeout -k 10 200 python3 -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu --no-parity > gpurun_out/big_ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/big_ab_$v.log; exit 1; }
  python3 -c "
import json
j = json.loads([l for l in open('gpurun_out/big_ab_$v.log') if l.startswith('{')][-1])
print('variant $v', 'step', j['ms_per_step'], 'scan', j['roofline']['avg_launch_ms'])"
  grep "^\[post\]" gpurun_out/big_ab_$v.log | tail -1
done
