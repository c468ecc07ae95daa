#!/bin/bash
# r04ad: k_report keyword bits as plain atomics: gate / parity GPU tests + configs[2]
set -o pipefail
mkdir -p gpurun_out/r04ad
export TMPDIR=/tmp
O=gpurun_out/r04ad
timeout -k 10 600 python -u -m pytest tests/test_gpu_stress.py tests/test_gpu_parity.py tests/test_gpu_fold.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['parity']['spot_mismatched_files'], d['parity']['planted_found'], d['parity']['decoys_found'])"
