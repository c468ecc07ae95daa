#!/bin/bash
# needs the ablation build: `make exp` here, then TSG_LIB_VARIANT=exp (exported below)
export TSG_LIB_VARIANT=exp
export TMPDIR=/tmp
for m in 0 1; do
TSG_REPORT_MODE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/rm_$m -o run -- python3 -u bench.py --gb 50 --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/rm_$m.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/rm_$m/run_kernel_stats.csv')):
    if 'k_report' in r['Name']: print($m, 'k_report', round(float(r['AverageNs'])/1e6,3))"
done
