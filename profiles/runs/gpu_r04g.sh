#!/bin/bash
# r04g: configs[2] line + timeline (gated DFA skip), configs[3] and configs[0] lines (pack workers)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_c2_r04g.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r04g.log; exit 1; }
tail -1 gpurun_out/bench_c2_r04g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['parity']['spot_mismatched_files'], d['parity']['planted_found'], d['parity']['decoys_found'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c2g -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c2g.log 2>&1 || { echo "c2 trace failed"; tail -20 gpurun_out/c2g.log; exit 1; }
python3 tools/timeline.py gpurun_out/c2g/run_kernel_trace.csv k_scan_fast 12 > gpurun_out/c2g/timeline.txt
awk '$2>0.05 || $3>0.03' gpurun_out/c2g/timeline.txt
timeout -k 10 400 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c3_r04g.log 2>&1 || { echo "bench c3 failed"; tail -20 gpurun_out/bench_c3_r04g.log; exit 1; }
tail -1 gpurun_out/bench_c3_r04g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_ms'], d['parity'] and {k: d['parity'][k] for k in ('planted','planted_found','decoys_found','spot_mismatched_files') if k in d['parity']})"
timeout -k 10 400 python -u bench.py --config 0 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c0_r04g.log 2>&1 || { echo "bench c0 failed"; tail -20 gpurun_out/bench_c0_r04g.log; exit 1; }
tail -1 gpurun_out/bench_c0_r04g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['host_ms'])"
