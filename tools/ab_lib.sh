#!/bin/bash
# Same-box A/B of the working tree's library against tools/build_alt.sh's
# (TSG_LIB_VARIANT=alt): bench.py per config, alternating, ROUNDS times.
# Usage: bash tools/ab_lib.sh <tag> "<configs>" [rounds] ["cur alt alt2 ..."]
set -o pipefail
TAG=$1; CFGS=$2; ROUNDS=${3:-2}; VARS=${4:-cur alt}
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq $ROUNDS); do
  for c in $CFGS; do
    for v in $VARS; do
      V=$v; [ $v = cur ] && V=""
      TSG_LIB_VARIANT=$V timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-parity \
        $BENCH_ARGS > $O/c${c}_${v}_$r.log 2>&1 || { echo "c$c $v failed"; tail -5 $O/c${c}_${v}_$r.log; exit 1; }
      python3 - $O/c${c}_${v}_$r.log "c$c $v r$r" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d.get("roofline") or {}
print(sys.argv[2], "ms", d["ms_per_step"], "scan", r.get("avg_launch_ms"), json.dumps(d.get("stages_ms")))
PY
    done
  done
done
