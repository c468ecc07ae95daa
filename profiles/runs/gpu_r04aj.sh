#!/bin/bash
# r04aj: phase-0 newline count grid under k_verify (exp, TSG_NL_BLOCKS_PER_CU): full grid | 4 | 2 | 1 blocks per CU
set -o pipefail
mkdir -p gpurun_out/r04aj
export TMPDIR=/tmp
O=gpurun_out/r04aj
export TSG_LIB_VARIANT=exp
for v in full 4 2 1 full; do
  if [ $v = full ]; then unset TSG_NL_BLOCKS_PER_CU; else export TSG_NL_BLOCKS_PER_CU=$v; fi
  timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --no-cpu > $O/c2_$v.log 2>&1 || { echo "variant $v failed"; tail -5 $O/c2_$v.log; exit 1; }
  tail -1 $O/c2_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms']['verify'], d['stages_ms']['lines'], d['parity']['spot_mismatched_files'], d['parity']['planted_found'])"
done
