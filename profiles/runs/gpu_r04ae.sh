#!/bin/bash
# r04ae: k_report with two interleaved events per lane: gate / parity GPU tests, configs[2], kernel stats
set -o pipefail
mkdir -p gpurun_out/r04ae
export TMPDIR=/tmp
O=gpurun_out/r04ae
timeout -k 10 600 python -u -m pytest tests/test_gpu_stress.py tests/test_gpu_parity.py tests/test_gpu_fold.py tests/test_gpu_analyzer.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['parity']['spot_mismatched_files'], d['parity']['planted_found'], d['parity']['decoys_found'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/c2trace -o run -- python3 -u bench.py --steps 4 --warmup 1 --no-cpu --no-parity > $O/c2trace.log 2>&1 || { echo "trace failed"; tail -5 $O/c2trace.log; exit 1; }
cp $O/c2trace/run_kernel_stats.csv $O/kernel_stats_c2.csv
grep -E "k_report|k_scan_fast" $O/kernel_stats_c2.csv | cut -c1-160
