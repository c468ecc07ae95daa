#!/bin/bash
# r04x: configs[3] staging A/B (exp build): pinned flags (non-coherent) and DMA chunk size
set -o pipefail
mkdir -p gpurun_out/r04x
export TMPDIR=/tmp
O=gpurun_out/r04x
export TSG_LIB_VARIANT=exp
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu > $O/c3_$tag.log 2>&1 || { echo "c3 $tag failed"; tail -20 $O/c3_$tag.log; return 1; }
  tail -1 $O/c3_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $tag', d['value'], d['ms_per_step'], d['host_ms'])"
}
run base TSG_X=0 && run nc TSG_STAGE_NC=1 && run chunk256 TSG_STAGE_CHUNK_MB=256 && run chunk16 TSG_STAGE_CHUNK_MB=16 && run base2 TSG_X=0
