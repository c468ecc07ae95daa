#!/bin/bash
# r03o: k_verify job-time profile on configs[4] (exp build, TSG_PROFILE_VERIFY):
# percentiles of job end times and durations, the slowest jobs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TSG_LIB_VARIANT=exp TSG_PROFILE_VERIFY=1 timeout -k 10 300 python3 -u bench.py --config 4 --steps 1 --warmup 1 --no-cpu --no-parity > gpurun_out/vprof_r03o.log 2> gpurun_out/vprof_r03o.err || { echo "vprof failed"; tail -20 gpurun_out/vprof_r03o.err; exit 1; }
grep -E "^\[verify\] (kernel|job ends|top-dur|top-steps)" gpurun_out/vprof_r03o.err | tail -40
