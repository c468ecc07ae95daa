#!/bin/bash
# r04v: side stream at the lowest priority (phase-0 newline count under k_verify): configs[2] x2 + timeline
set -o pipefail
mkdir -p gpurun_out/r04v
export TMPDIR=/tmp
O=gpurun_out/r04v
for r in 1 2; do
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_c2_$r.log 2>&1 || { echo "bench c2 failed"; tail -20 $O/bench_c2_$r.log; exit 1; }
tail -1 $O/bench_c2_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['parity']['spot_mismatched_files'], d['parity']['planted_found'], d['parity']['decoys_found'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/c2trace -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu --no-parity > $O/c2trace.log 2>&1 || { echo "c2 trace failed"; tail -20 $O/c2trace.log; exit 1; }
python3 tools/timeline.py $O/c2trace/run_kernel_trace.csv k_scan_fast 12 > $O/timeline_c2.txt
tail -1 $O/timeline_c2.txt
