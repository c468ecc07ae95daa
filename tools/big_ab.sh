#!/bin/bash
# Timing bounds of k_scan_big on configs[4] (ablation build, `make exp`):
# TSG_BIG_VARIANT "<mode>[x<chains>][v<ring>]" (engine.hip big_group): mode 0 = product walk,
# 1 = byte class from ALU instead of LDS, 2 = dense rows only (no cold-state
# records), 3 = both, 4 = one event ballot per 16 bytes, 8 = dense reads of all
# chains issued before cold walks; x2 = two chains per lane.  Modes 1-3 give
# wrong results: only their scan time (HIP events, roofline.avg_launch_ms)
# is read.
export TSG_LIB_VARIANT=exp
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 2 3 4 4v4 0x2v2 8x2v2 12x2v2 0x2v4 8x2v4; do
  export TSG_BIG_VARIANT=$v
  timeout -k 10 300 python3 -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu --no-parity > gpurun_out/big_ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/big_ab_$v.log; exit 1; }
  python3 -c "
import json
j = json.loads([l for l in open('gpurun_out/big_ab_$v.log') if l.startswith('{')][-1])
print('variant $v', 'step', j['ms_per_step'], 'scan', j['roofline']['avg_launch_ms'])"
done
