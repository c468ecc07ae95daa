#!/bin/bash
# needs the ablation build: `make exp` here, then TSG_LIB_VARIANT=exp (exported below)
export TSG_LIB_VARIANT=exp
# Per k_scan_fast shape: kernel time (trace) and HBM read bytes (FETCH_SIZE pass) on an 8 GB corpus.
set -o pipefail
export TMPDIR=/tmp
for v in ${VARIANTS:-1x8 1x4 2x2}; do
  export TSG_FAST_VARIANT=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abf_$v/t -o run -- python3 -u bench.py --gb 8 --steps 2 --warmup 1 --no-cpu --no-parity > gpurun_out/abf_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS -f csv -d gpurun_out/abf_$v/f -o run -- python3 -u bench.py --gb 8 --steps 1 --warmup 0 --no-cpu --no-parity >> gpurun_out/abf_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 - $v <<'PY'
import csv, sys, collections
v = sys.argv[1]
t = [r for r in csv.DictReader(open(f"gpurun_out/abf_{v}/t/run_kernel_stats.csv")) if "k_scan_fast" in r["Name"] or "k_report" in r["Name"]]
c = collections.defaultdict(float)
for r in csv.DictReader(open(f"gpurun_out/abf_{v}/f/run_counter_collection.csv")):
    if "k_scan_fast" in r["Kernel_Name"]:
        c[r["Counter_Name"]] += float(r["Counter_Value"])
print(v, [(r["Name"].split("::")[1].split("(")[0], round(float(r["AverageNs"]) / 1e6, 3)) for r in t],
      "fetch_GB_corr", round(c["FETCH_SIZE"] * 2048 / 1e9, 2), "conf/idx", round(c["SQ_LDS_BANK_CONFLICT"] / max(1, c["SQ_LDS_IDX_ACTIVE"]), 3),
      "lds_instr", c["SQ_INSTS_LDS"], "wait_frac", round(c["SQ_WAIT_ANY"] / max(1, c["SQ_WAVE_CYCLES"]), 3), flush=True)
PY
done
