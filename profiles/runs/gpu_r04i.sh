#!/bin/bash
# r04i: configs[4] k_verify stage with / without DFA run acceleration (exp build)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu --no-parity > gpurun_out/ab4_$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/ab4_$name.log; return 1; }
  grep '^{' gpurun_out/ab4_$name.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'], d['stages_ms']['verify'])"
}
run exp TSG_LIB_VARIANT=exp && run exp_noaccel TSG_LIB_VARIANT=exp TSG_NO_ACCEL=1 && run exp2 TSG_LIB_VARIANT=exp && run exp_noaccel2 TSG_LIB_VARIANT=exp TSG_NO_ACCEL=1
