#!/bin/bash
# Kernel trace + stats of the configs[2] bench (no parity legs): per-kernel time.
# Usage (GPU box, repo root): bash tools/trace.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-trace}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-parity "$@" > $OUT/bench.log 2>&1 || { echo "trace failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$OUT/trace/run_kernel_stats.csv')))
for r in rows[:25]: print(r['Name'][:70].ljust(70), r['Calls'], '%.3f'%(float(r['AverageNs'])/1e6), '%.3f'%(float(r['TotalDurationNs'])/1e6))
"
