#!/bin/bash
# r04z: configs[3] per-layer phase times after the path-DFA Required
set -o pipefail
mkdir -p gpurun_out/r04z
export TMPDIR=/tmp
O=gpurun_out/r04z
TSG_C3_TRACE=1 timeout -k 10 400 python -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-parity > $O/c3.log 2> $O/c3.err || { echo "c3 failed"; tail -20 $O/c3.err; exit 1; }
tail -8 $O/c3.err
tail -1 $O/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['ms_per_step'], d['host_ms'])"
