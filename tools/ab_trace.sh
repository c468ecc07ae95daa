#!/bin/bash
# Kernel-trace A/B of exp-build switches on configs[2] (or BENCH_ARGS):
# per variant (space-separated "ENV=V[,ENV2=V2]" items, "-" = none) one
# rocprofv3 --kernel-trace run of the bench, then the last step's timeline
# (tools/timeline.py) and the key kernels' durations in that step.
# Usage: bash tools/ab_trace.sh <tag> "<variant> ..."
export TSG_LIB_VARIANT=exp
set -o pipefail
export TMPDIR=/tmp
TAG=$1; VARS=$2
O=gpurun_out/$TAG
mkdir -p $O
i=0
for v in $VARS; do
  i=$((i + 1))
  E=""
  [ "$v" != "-" ] && E=$(echo "$v" | tr ',' ' ')
  env $E timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/t$i -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-parity $BENCH_ARGS > $O/t$i.log 2>&1 \
    || { echo "variant $v failed"; tail -5 $O/t$i.log; exit 1; }
  python3 tools/timeline.py $O/t$i/run_kernel_trace.csv > $O/timeline_$i.txt
  python3 - "$O/timeline_$i.txt" "$O/t$i.log" "$v" <<'PY'
import collections, json, sys
tl, log, v = sys.argv[1:4]
agg = collections.Counter()
span = None
for line in open(tl):
    p = line.split(None, 3)
    if line.startswith("span"):
        span = line.split()[1]
        continue
    try:
        d = float(p[1])
    except (ValueError, IndexError):
        continue
    k = p[3].split("<")[0].strip()
    agg["rocprim" if "rocprim" in k else k] += d
d = json.loads([l for l in open(log) if l.startswith("{")][-1])
keys = ["k_scan_fast", "k_scan_lines", "k_scan_big", "k_report", "k_path_gate", "k_expand", "k_verify", "k_captures",
        "k_nl_spans", "k_find_spans", "rocprim", "__amd_rocclr_copyBuffer"]
print(v, "step", d["ms_per_step"], "span", span, {k: round(agg[k], 3) for k in keys if agg[k]})
PY
done
