#!/bin/bash
# r04q: flat cold records (one record + the dense ancestor's row per cold byte, branch-free for the wave):
# big-path GPU tests, configs[4] x2, exp bounds 24x2v2 (test+branch only) for reference
set -o pipefail
mkdir -p gpurun_out/r04q
export TMPDIR=/tmp
O=gpurun_out/r04q
timeout -k 10 600 python -u -m pytest tests/test_gpu_big_global.py tests/test_gpu_stress.py tests/test_gpu_verify_split.py tests/test_gpu_censor_big.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu > $O/bench_c4_$r.log 2>&1 || { echo "bench c4 failed"; tail -20 $O/bench_c4_$r.log; exit 1; }
tail -1 $O/bench_c4_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['parity']['stress_mismatched_files'], d['parity']['spot_mismatched_files'])"
done
export TSG_LIB_VARIANT=exp
TSG_BIG_VARIANT=24x2v2 timeout -k 10 300 python3 -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu --no-parity > $O/big_24.log 2>&1 || { echo "variant failed"; tail -5 $O/big_24.log; exit 1; }
tail -1 $O/big_24.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('24x2v2', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
