#!/bin/bash
# r04p: k_scan_big bounds after the r04m dense step (exp build, wrong-result bounds marked):
# 8x2v2 product | 24x2v2 cold test + branch, no cold walk (bound) | 25x2v2 same + class from ALU | 2x2v2 dense only | 9x2v2 class ALU
set -o pipefail
mkdir -p gpurun_out/r04p
export TMPDIR=/tmp
O=gpurun_out/r04p
export TSG_LIB_VARIANT=exp
for v in 8x2v2 24x2v2 25x2v2 2x2v2 9x2v2; do
  TSG_BIG_VARIANT=$v timeout -k 10 300 python3 -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu --no-parity > $O/big_$v.log 2>&1 || { echo "variant $v failed"; tail -5 $O/big_$v.log; exit 1; }
  tail -1 $O/big_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['counts']['events'])"
done
