#!/bin/bash
# r04w: PMC passes for configs[2] and configs[4] on the round-4 kernels; configs[3] A/B of the staging DMA over
# one vs two streams (exp build, TSG_DMA_STREAMS)
set -o pipefail
mkdir -p gpurun_out/r04w
export TMPDIR=/tmp
O=gpurun_out/r04w
bash tools/pmc.sh r04w_c2 2 && bash tools/pmc.sh r04w_c4 4 || exit 1
for v in 1 2 1 2; do
  TSG_LIB_VARIANT=exp TSG_DMA_STREAMS=$v timeout -k 10 400 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu > $O/c3_dma$v.log 2>&1 || { echo "c3 $v failed"; tail -20 $O/c3_dma$v.log; exit 1; }
  tail -1 $O/c3_dma$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 dma$v', d['value'], d['ms_per_step'], d['host_ms'])"
done
