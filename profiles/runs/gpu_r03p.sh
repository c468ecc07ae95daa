#!/bin/bash
# r03p: configs[2] kernel timeline (rocprofv3 kernel trace of the last step).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c2p -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c2p.log 2>&1 || { echo "c2 trace failed"; tail -20 gpurun_out/c2p.log; exit 1; }
python3 tools/timeline.py gpurun_out/c2p/run_kernel_trace.csv k_scan_fast 12 > gpurun_out/c2p/timeline.txt
cat gpurun_out/c2p/timeline.txt
