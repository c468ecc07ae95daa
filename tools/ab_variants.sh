#!/bin/bash
# needs the ablation build: `make exp` here, then TSG_LIB_VARIANT=exp (exported below)
export TSG_LIB_VARIANT=exp
# A/B the k_scan_fast shapes (TSG_FAST_VARIANT=chains x vectors) on the GPU box:
# parity tests once, then per variant a bench line (with parity properties)
# under a rocprofv3 kernel trace, printing per-kernel average times.
set -o pipefail
export TMPDIR=/tmp
[ -n "$SKIP_CHECK" ] || bash tools/gpu_run.sh ab_check pytest smoke || exit 1
GB=${GB:-20}
for v in ${VARIANTS:-1x8 1x4 2x4}; do
  TSG_FAST_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ab_$v -o run -- python3 -u bench.py --gb $GB --steps 3 --warmup 1 --no-cpu > gpurun_out/ab_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, json, sys
v = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/ab_{v}.log") if l.startswith("{")][-1])
ks = {}
for r in csv.DictReader(open(f"gpurun_out/ab_{v}/run_kernel_stats.csv")):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    if n.startswith("k_"):
        ks[n] = round(float(r["AverageNs"]) / 1e6, 3)
print(v, "value", d["value"], "stages", d["stages_ms"], "counts", d["counts"], "kernels_ms", ks,
      "parity_ok", d["parity"]["planted"] == d["parity"]["planted_found"] and d["parity"]["spot_mismatched_files"] == 0)
PY
done
