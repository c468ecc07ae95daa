#!/bin/bash
# r04m: k_scan_big dense step (mad24 offsets, one wave-uniform cold test, LDS/global cold records): GPU suite, configs[4],
# exp A/B of the LDS cold-record floor (TSG_BIG_COLD_LDS)
set -o pipefail
mkdir -p gpurun_out/r04m
export TMPDIR=/tmp
O=gpurun_out/r04m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu > $O/bench_c4.log 2>&1 || { echo "bench c4 failed"; tail -20 $O/bench_c4.log; exit 1; }
tail -1 $O/bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['parity']['stress_mismatched_files'], d['parity']['spot_mismatched_files'])"
export TSG_LIB_VARIANT=exp
for v in 1024 2048 4096 100000; do
  TSG_BIG_COLD_LDS=$v timeout -k 10 300 python3 -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu > $O/cold_$v.log 2>&1 || { echo "variant $v failed"; tail -5 $O/cold_$v.log; exit 1; }
  tail -1 $O/cold_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cold_lds $v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['parity']['stress_mismatched_files'], d['parity']['spot_mismatched_files'])"
done
