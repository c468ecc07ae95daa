#!/bin/bash
# r04n: k_scan_big bounds after the r04m dense step (exp build, wrong-result bounds marked):
# 8x2v2 product | 9x2v2 class from ALU (bound) | 2x2v2 dense rows only (bound) | 3x2v2 both (bound)
set -o pipefail
mkdir -p gpurun_out/r04n
export TMPDIR=/tmp
O=gpurun_out/r04n
export TSG_LIB_VARIANT=exp
for v in 8x2v2 9x2v2 2x2v2 3x2v2 8x2v2; do
  TSG_BIG_VARIANT=$v timeout -k 10 300 python3 -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu --no-parity > $O/big_$v.log 2>&1 || { echo "variant $v failed"; tail -5 $O/big_$v.log; exit 1; }
  tail -1 $O/big_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['counts']['events'])"
done
