#!/bin/bash
# r04t: lazy newline counts (fast path only), phase 0 on the side stream under k_verify:
# full GPU suite, configs[2] (parity + cpu baseline) and configs[4]
set -o pipefail
mkdir -p gpurun_out/r04t
export TMPDIR=/tmp
O=gpurun_out/r04t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['cpu_baseline']['value'], d['parity']['spot_mismatched_files'], d['parity']['planted_found'], d['parity']['decoys_found'])"
timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu > $O/bench_c4.log 2>&1 || { echo "bench c4 failed"; tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['parity']['stress_mismatched_files'], d['parity']['spot_mismatched_files'])"
