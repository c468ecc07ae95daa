#!/bin/bash
# r04h: k_verify on configs[2]: product vs exp without run acceleration, and the per-job profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu --no-parity > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/ab_$name.log; return 1; }
  grep '^{' gpurun_out/ab_$name.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'], d['stages_ms']['verify'])"
}
run prod X=1 && run exp TSG_LIB_VARIANT=exp && run exp_noaccel TSG_LIB_VARIANT=exp TSG_NO_ACCEL=1 && \
run exp_prof TSG_LIB_VARIANT=exp TSG_PROFILE_VERIFY=1 && grep -A25 "\[verify\]" gpurun_out/ab_exp_prof.log | tail -40
