#!/bin/bash
# A/B the verify shapes (split search + k_captures vs one inline kernel) at 50 GB.
set -o pipefail
export TMPDIR=/tmp
for v in split inline; do
  if [ $v = split ]; then export TSG_VERIFY_SPLIT=1; else unset TSG_VERIFY_SPLIT; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abv_$v -o run -- python3 -u bench.py --gb ${GB:-50} --steps 3 --warmup 1 --no-cpu > gpurun_out/abv_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/abv_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, json, sys
v = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/abv_{v}.log") if l.startswith("{")][-1])
ks = {}
for r in csv.DictReader(open(f"gpurun_out/abv_{v}/run_kernel_stats.csv")):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    if n.startswith("k_v") or n.startswith("k_c"):
        ks[n] = round(float(r["AverageNs"]) / 1e6, 3)
print(v, "value", d["value"], "verify", d["stages_ms"]["verify"], ks,
      "parity_ok", d["parity"]["planted"] == d["parity"]["planted_found"] and d["parity"]["spot_mismatched_files"] == 0)
PY
done
