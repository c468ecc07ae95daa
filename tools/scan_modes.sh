#!/bin/bash
# needs the ablation build: `make exp` here, then TSG_LIB_VARIANT=exp (exported below)
export TSG_LIB_VARIANT=exp
# Timing-only ablation of k_scan_fast (TSG_SCAN_MODE bits: 1 = no events, 2 = no newline count,
# 4 = loads from the first MiB only (L2-resident), so HBM is out of the picture).
set -o pipefail
export TMPDIR=/tmp
for m in ${MODES:-0 1 2 3 4 7}; do
  TSG_SCAN_MODE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sm_$m -o run -- python3 -u bench.py --gb 20 --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/sm_$m.log 2>&1 || { echo "mode $m failed"; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/sm_$m/run_kernel_stats.csv')):
    if 'k_scan_fast' in r['Name']: print($m, r['Name'].split('::')[1].split('(')[0], round(float(r['AverageNs'])/1e6, 3))"
done
