#!/bin/bash
# Generic A/B of exp-build switches on one bench config, alternating within
# one gpurun call (box-to-box spread is larger than most single changes).
# Usage: bash tools/ab_env.sh <tag> "<envA>" "<envB>" [reps] [bench args]
#   e.g. bash tools/ab_env.sh r05b "TSG_FUSE=0" "TSG_FUSE=1" 2 "--config 2"
# Each run: step and scan-kernel time, stage times, counts, parity properties
# (the first rep of each variant with the oracle spot checks).
export TSG_LIB_VARIANT=exp
set -o pipefail
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; REPS=${4:-2}; ARGS=${5:-}
O=gpurun_out/$TAG
mkdir -p $O
for rep in $(seq 1 $REPS); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    extra="--no-parity"
    [ $rep = 1 ] && extra=""
    env $E timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu $extra $ARGS > $O/ab_${v}_$rep.log 2>&1 \
      || { echo "$v ($E) failed"; tail -5 $O/ab_${v}_$rep.log; exit 1; }
    python3 - "$O/ab_${v}_$rep.log" "$v" "$E" "$rep" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
p = d.get("parity") or {}
r = d.get("roofline") or {}
print(sys.argv[2], sys.argv[3], "rep", sys.argv[4], "value", d["value"], "step", d["ms_per_step"], "scan",
      r.get("avg_launch_ms"), "stages", d.get("stages_ms"), "counts", d.get("counts"),
      "parity", {k: p.get(k) for k in ("planted", "planted_found", "decoys_found", "spot_mismatched_files",
                                       "stress_mismatched_files") if k in p})
PY
  done
done
