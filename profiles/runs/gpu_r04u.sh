#!/bin/bash
# r04u: configs[2] kernel timeline after the lazy newline counts (rocprofv3 kernel trace, last step)
set -o pipefail
mkdir -p gpurun_out/r04u
export TMPDIR=/tmp
O=gpurun_out/r04u
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/c2trace -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu --no-parity > $O/c2trace.log 2>&1 || { echo "c2 trace failed"; tail -20 $O/c2trace.log; exit 1; }
python3 tools/timeline.py $O/c2trace/run_kernel_trace.csv k_scan_fast 12 > $O/timeline_c2.txt
cp $O/c2trace/run_kernel_stats.csv $O/kernel_stats_c2.csv
tail -1 $O/timeline_c2.txt
