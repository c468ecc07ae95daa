#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box from the repo root):
#   1. kernel trace + stats of the default bench workload (50 GB, configs[2])
#   2. PMC pass: FETCH_SIZE (HBM read traffic) per dispatch
#   3. PMC pass: SQ counters (LDS bank conflicts, VALU/LDS instruction mix, waits)
# Usage: bash tools/profile.sh <tag> [gb] [config]   (config 4: the k_scan_big stress workload)
set -o pipefail
TAG=${1:-r01}
GB=${2:-50}
CFG=${3:-2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --config $CFG --gb $GB --steps 3 --warmup 1 --no-cpu --no-parity"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $B > $OUT/trace_bench.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace_bench.log; exit 1; }
tail -1 $OUT/trace_bench.log
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- python3 bench.py --config $CFG --gb $GB --steps 1 --warmup 0 --no-cpu --no-parity > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/fetch.log; exit 1; }
grep '^{' $OUT/fetch.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['roofline']['algorithmic_bytes_per_launch'])" > $OUT/alg_bytes.txt
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -f csv -d $OUT/sq -o run -- python3 bench.py --config $CFG --gb 8 --steps 2 --warmup 0 --no-cpu --no-parity > $OUT/sq.log 2>&1 || { echo "sq pass failed"; tail -20 $OUT/sq.log; exit 1; }
find $OUT -name "*.csv" | head -20
