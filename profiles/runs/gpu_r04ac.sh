#!/bin/bash
# r04ac: k_report A/B (exp build, TSG_REPORT_MODE): 0 product | 2 keyword atomicOr without the read | 1 no file lookup (bound, wrong) | 3 both
set -o pipefail
mkdir -p gpurun_out/r04ac
export TMPDIR=/tmp
O=gpurun_out/r04ac
export TSG_LIB_VARIANT=exp
for m in 0 2 1 3 0; do
  TSG_REPORT_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/m$m -o run -- python3 -u bench.py --steps 4 --warmup 1 --no-cpu --no-parity > $O/m$m.log 2>&1 || { echo "mode $m failed"; tail -5 $O/m$m.log; exit 1; }
  python3 - "$O/m$m/run_kernel_stats.csv" "$m" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("k_report", "k_expand")):
        print("mode", sys.argv[2], r["Name"][:20], r["AverageNs"])
PY
done
