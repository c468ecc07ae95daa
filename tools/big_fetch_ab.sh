#!/bin/bash
# k_scan_big load shapes (TSG_BIG_VARIANT, exp build) on configs[4]: per
# variant one FETCH_SIZE pass (HBM/fabric bytes per launch, x2 gfx950
# correction) and one kernel-trace pass (average launch time), each under its
# own kill timer.  Usage: bash tools/big_fetch_ab.sh <tag> "<variant> ..."
# ("default" = the product shape, "L1" / "L2" = k_scan_lines with 2 / 1 chains).
export TSG_LIB_VARIANT=exp
set -o pipefail
export TMPDIR=/tmp
TAG=$1; VARS=${2:-"default"}
O=gpurun_out/$TAG
mkdir -p $O
ARGS="--config 4 --steps 2 --warmup 1 --no-cpu --no-parity"
for v in $VARS; do
  unset TSG_BIG_VARIANT TSG_BIG_LINES
  case "$v" in
    default) ;;
    L*) export TSG_BIG_LINES=${v#L} ;;  # k_scan_lines: L1 = 2 chains, L2 = 1 chain
    *) export TSG_BIG_VARIANT=$v ;;
  esac
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch_$v -o run -- python3 bench.py $ARGS > $O/fetch_$v.log 2>&1 \
    || { echo "fetch $v failed"; tail -5 $O/fetch_$v.log; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_$v -o run -- python3 bench.py $ARGS > $O/trace_$v.log 2>&1 \
    || { echo "trace $v failed"; tail -5 $O/trace_$v.log; exit 1; }
  python3 - "$O" "$v" <<'PY'
import csv, glob, sys
o, v = sys.argv[1], sys.argv[2]
fs = [float(r["Counter_Value"]) for f in glob.glob(f"{o}/fetch_{v}/**/*counter_collection.csv", recursive=True)
      for r in csv.DictReader(open(f)) if ("k_scan_big" in r["Kernel_Name"] or "k_scan_lines" in r["Kernel_Name"]) and r["Counter_Name"] == "FETCH_SIZE"]
ts = [r for f in glob.glob(f"{o}/trace_{v}/**/*kernel_stats.csv", recursive=True) for r in csv.DictReader(open(f))
      if "k_scan_big" in r["Name"] or "k_scan_lines" in r["Name"]]
fetch = sum(fs) / len(fs) * 1024 * 2 / 1e9 if fs else None
ms = float(ts[0]["AverageNs"]) / 1e6 if ts else None
print(f"{v}: k_scan_big fetch {fetch:.2f} GB/launch (x2 corrected), avg {ms:.3f} ms, launches {len(fs)}")
PY
done
