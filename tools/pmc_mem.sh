#!/bin/bash
# Memory-hierarchy counters of the scan kernel (one rocprofv3 --pmc pass per
# counter group, each under its own kill timer): L2 requests / hits / misses,
# L1->L2 read requests and L1 accesses, texture-addresser busy.
# Usage: bash tools/pmc_mem.sh [gb]   (writes gpurun_out/pmc_mem/<pass>/)
set -o pipefail
export TMPDIR=/tmp
GB=${1:-8}
OUT=gpurun_out/pmc_mem
mkdir -p $OUT
B="bench.py --gb $GB --steps 1 --warmup 0 --no-cpu --no-parity"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d $OUT/$name -o run -- python3 $B > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; return 1; }
}
pass tcc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum && \
pass tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum && \
pass fetch FETCH_SIZE && \
pass ta TA_TA_BUSY_sum TA_BUFFER_LOAD_WAVEFRONTS_sum
python3 - <<'PY'
import csv, glob, collections
for fn in sorted(glob.glob("gpurun_out/pmc_mem/*/run_counter_collection.csv")):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(fn)):
        if "k_scan_fast" in r["Kernel_Name"] or "k_report" in r["Kernel_Name"]:
            k = "scan" if "k_scan_fast" in r["Kernel_Name"] else "report"
            d[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(d.items()):
        print(fn.split("/")[-2], k, c, sum(v) / len(v))
PY
