#!/bin/bash
# Counter passes on the scan kernels only (small corpus): kernel trace + 2 SQ passes + FETCH_SIZE.
# Usage: bash tools/prof_scan.sh <tag> [gb]
set -o pipefail
TAG=${1:-scan}; GB=${2:-8}
OUT=gpurun_out/prof_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
B="bench.py --gb $GB --steps 2 --warmup 0 --no-cpu --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || { echo trace failed; tail -5 $OUT/trace.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -f csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1 || { echo sq failed; tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -f csv -d $OUT/sq2 -o run -- python3 $B > $OUT/sq2.log 2>&1 || { echo sq2 failed; tail -5 $OUT/sq2.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1 || { echo fetch failed; tail -5 $OUT/fetch.log; exit 1; }
python3 tools/prof_summary.py $OUT $OUT/summary | grep -E "k_scan|k_report|k_verify|k_path|k_expand"
