#!/bin/bash
# configs[4] diagnostics: a rocprofv3 kernel summary + trace of the product
# library, then per-job / per-rule k_verify times and the host post split (exp
# build, TSG_PROFILE_VERIFY).  Usage (repo root, GPU box): bash tools/c4_verify_prof.sh [GB] [tag]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GB=${1:-10}
TAG=${2:-c4}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_prof -o run -- python3 -u bench.py --config 4 \
  --gb "$GB" --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof run failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_prof.log
TSG_LIB_VARIANT=exp TSG_PROFILE_VERIFY=1 timeout -k 10 400 python3 -u bench.py --config 4 --gb "$GB" --steps 1 --warmup 0 \
  --no-cpu --no-parity > gpurun_out/${TAG}_vprof.log 2> gpurun_out/${TAG}_vprof.err || { echo "vprof run failed"; tail -20 gpurun_out/${TAG}_vprof.err; exit 1; }
tail -1 gpurun_out/${TAG}_vprof.log
grep "\[post\]" gpurun_out/${TAG}_vprof.err | tail -2
