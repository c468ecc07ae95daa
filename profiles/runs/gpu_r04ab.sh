#!/bin/bash
# r04ab: round-4 tree after the k_scan_big, lazy newline and configs[3] changes: GPU suite, smoke, configs[2] (cpu baseline + parity), c2 kernel trace, configs[4], [0], [1], [3]
set -o pipefail
mkdir -p gpurun_out/r04ab
export TMPDIR=/tmp
O=gpurun_out/r04ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
timeout -k 10 400 python -u bench.py > $O/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['cpu_baseline']['value'], d['parity']['spot_mismatched_files'], d['parity']['planted_found'], d['parity']['decoys_found'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/c2trace -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu --no-parity > $O/c2trace.log 2>&1 || { echo "c2 trace failed"; tail -20 $O/c2trace.log; exit 1; }
python3 tools/timeline.py $O/c2trace/run_kernel_trace.csv k_scan_fast 12 > $O/timeline_c2.txt
tail -1 $O/timeline_c2.txt
timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu > $O/bench_c4.log 2>&1 || { echo "bench c4 failed"; tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['parity']['stress_mismatched_files'], d['parity']['spot_mismatched_files'])"
timeout -k 10 400 python -u bench.py --config 0 --steps 5 --warmup 2 > $O/bench_c0.log 2>&1 || { echo "bench c0 failed"; tail -20 $O/bench_c0.log; exit 1; }
tail -1 $O/bench_c0.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c0', d['value'], d['ms_per_step'], d['cpu_baseline'] and d['cpu_baseline']['value'])"
timeout -k 10 400 python -u bench.py --config 1 --steps 10 --warmup 3 --no-cpu > $O/bench_c1.log 2>&1 || { echo "bench c1 failed"; tail -20 $O/bench_c1.log; exit 1; }
tail -1 $O/bench_c1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['value'], d['ms_per_step'])"
timeout -k 10 400 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu > $O/bench_c3.log 2>&1 || { echo "bench c3 failed"; tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/c4trace -o run -- python3 -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu --no-parity > $O/c4trace.log 2>&1 || { echo "c4 trace failed"; tail -20 $O/c4trace.log; exit 1; }
cp $O/c4trace/run_kernel_stats.csv $O/kernel_stats_c4.csv
python3 tools/timeline.py $O/c4trace/run_kernel_trace.csv k_scan_big 12 > $O/timeline_c4.txt
tail -1 $O/timeline_c4.txt
