#!/bin/bash
# needs the ablation build: `make exp` here, then TSG_LIB_VARIANT=exp (exported below)
export TSG_LIB_VARIANT=exp
# Ablation of k_scan_big (configs[4]) by TSG_REPORT_MODE: 0 normal, 8 no inline
# reports, 16 cold states answered by the root row, 24 both.  Kernel time from
# rocprofv3; modes != 0 give wrong findings (timing only, no parity).
set -o pipefail
export TMPDIR=/tmp
for m in ${MODES:-0 8 16 24}; do
  TSG_REPORT_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/big_$m -o run -- python3 -u bench.py --config 4 --gb 10 --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/big_$m.log 2>&1 || { echo "mode $m failed"; tail -5 gpurun_out/big_$m.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/big_$m/run_kernel_stats.csv')):
    if 'k_scan_big' in r['Name']: print($m, 'k_scan_big ms', round(float(r['AverageNs'])/1e6, 3))"
done
