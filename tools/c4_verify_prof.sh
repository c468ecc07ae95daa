#!/bin/bash
# configs[4] verify diagnostics: per-job / per-rule k_verify times (exp build,
# TSG_PROFILE_VERIFY) plus a rocprofv3 kernel summary of the same workload.
# Usage (repo root, GPU box): bash tools/c4_verify_prof.sh [GB]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GB=${1:-10}
TSG_LIB_VARIANT=exp TSG_PROFILE_VERIFY=1 timeout -k 10 400 python3 -u bench.py --config 4 --gb "$GB" --steps 1 --warmup 0 \
  --no-cpu --no-parity > gpurun_out/c4_vprof.log 2> gpurun_out/c4_vprof.err || { echo "vprof run failed"; tail -20 gpurun_out/c4_vprof.err; exit 1; }
tail -1 gpurun_out/c4_vprof.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c4_prof -o run -- python3 -u bench.py --config 4 \
  --gb "$GB" --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c4_prof.log 2>&1 || { echo "prof run failed"; tail -20 gpurun_out/c4_prof.log; exit 1; }
tail -1 gpurun_out/c4_prof.log
