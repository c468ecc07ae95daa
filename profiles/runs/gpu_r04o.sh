#!/bin/bash
# r04o: global cold records under test (floor 0) + the big-path GPU tests; configs[4] product (floor 4096) x2
set -o pipefail
mkdir -p gpurun_out/r04o
export TMPDIR=/tmp
O=gpurun_out/r04o
timeout -k 10 600 python -u -m pytest tests/test_gpu_big_global.py tests/test_gpu_stress.py tests/test_gpu_verify_split.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu > $O/bench_c4_$r.log 2>&1 || { echo "bench c4 failed"; tail -20 $O/bench_c4_$r.log; exit 1; }
tail -1 $O/bench_c4_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['parity']['stress_mismatched_files'], d['parity']['spot_mismatched_files'])"
done
