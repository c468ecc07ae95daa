#!/bin/bash
# r03l: GPU suite, configs[4] line + timeline (frequency-ordered k_scan_big
# states, 16-byte Match prefix sort), configs[2] line, k_scan_big A/B
# (exp build: breadth-first numbering vs frequency order, two chains).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_r03l.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r03l.log; exit 1; }
tail -2 gpurun_out/pytest_r03l.log
timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 2 > gpurun_out/bench_c4_r03l.log 2>&1 || { echo "bench c4 failed"; tail -20 gpurun_out/bench_c4_r03l.log; exit 1; }
tail -1 gpurun_out/bench_c4_r03l.log | cut -c1-1500
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c4l -o run -- python3 -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c4l.log 2>&1 || { echo "c4 trace failed"; tail -20 gpurun_out/c4l.log; exit 1; }
python3 tools/timeline.py gpurun_out/c4l/run_kernel_trace.csv k_scan_big 12 > gpurun_out/c4l/timeline.txt
awk '$2>0.05 || $3>0.05' gpurun_out/c4l/timeline.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_c2_r03l.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r03l.log; exit 1; }
tail -1 gpurun_out/bench_c2_r03l.log | cut -c1-700
export TSG_LIB_VARIANT=exp
for v in bfs:0 freq:0 freq:8x2v2 freq:2; do
  order=${v%%:*}; export TSG_BIG_VARIANT=${v#*:}
  if [ $order = bfs ]; then export TSG_BIG_BFS=1; else unset TSG_BIG_BFS; fi
  timeout -k 10 200 python3 -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu --no-parity > gpurun_out/big_ab_l_${order}_${TSG_BIG_VARIANT}.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/big_ab_l_${order}_${TSG_BIG_VARIANT}.log; exit 1; }
  python3 -c "
import json
j = json.loads([l for l in open('gpurun_out/big_ab_l_${order}_${TSG_BIG_VARIANT}.log') if l.startswith('{')][-1])
print('variant $v', 'step', j['ms_per_step'], 'scan', j['roofline']['avg_launch_ms'])"
  grep "^\[post\]" gpurun_out/big_ab_l_${order}_${TSG_BIG_VARIANT}.log | tail -1
done
