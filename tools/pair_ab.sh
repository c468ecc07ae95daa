#!/bin/bash
# A/B of k_scan_fast's root pair table (TSG_FAST_VARIANT=pair, fstep2) against
# the single-step walk, alternating, on the 50 GB configs[2] corpus: step and
# k_scan_fast time (HIP events) per run, parity properties of each variant.
# Needs the ablation build (`make exp`).
export TSG_LIB_VARIANT=exp
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in base pair; do
    if [ $v = pair ]; then export TSG_FAST_VARIANT=pair; else unset TSG_FAST_VARIANT; fi
    extra="--no-parity"
    [ $rep = 1 ] && extra=""
    timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu $extra > gpurun_out/pair_${v}_$rep.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/pair_${v}_$rep.log; exit 1; }
    python3 -c "
import json
j = json.loads([l for l in open('gpurun_out/pair_${v}_$rep.log') if l.startswith('{')][-1])
p = j['parity'] or {}
print('$v', $rep, 'value', j['value'], 'step', j['ms_per_step'], 'scan', j['roofline']['avg_launch_ms'], 'events', j['counts']['events'],
      'planted', p.get('planted_found'), '/', p.get('planted'), 'decoys', p.get('decoys_found'), 'spot_bad', p.get('spot_mismatched_files'))"
  done
done
