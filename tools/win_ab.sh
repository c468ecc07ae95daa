#!/bin/bash
# needs the ablation build: `make exp` here, then TSG_LIB_VARIANT=exp (exported below)
export TSG_LIB_VARIANT=exp
# A/B of k_scan_fast's event-check window (TSG_EVENT_WIN = 8-byte groups per
# wave-level check), kernel time from rocprofv3 + bench parity properties.
set -o pipefail
export TMPDIR=/tmp
for w in ${WINS:-1 2 4}; do
  TSG_EVENT_WIN=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/win_$w -o run -- python3 -u bench.py --gb 20 --steps 3 --warmup 1 --no-cpu > gpurun_out/win_$w.log 2>&1 || { echo "win $w failed"; tail -5 gpurun_out/win_$w.log; exit 1; }
  python3 -c "
import csv, json
for r in csv.DictReader(open('gpurun_out/win_$w/run_kernel_stats.csv')):
    if 'k_scan_fast' in r['Name']: print($w, r['Name'].split('::')[1].split('(')[0], round(float(r['AverageNs'])/1e6, 3))
j = json.loads([l for l in open('gpurun_out/win_$w.log') if l.startswith('{')][-1])
print('  value', j['value'], 'parity', j['parity'])"
done
