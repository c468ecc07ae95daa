#!/bin/bash
# Per-kernel rocprofv3 counters for one bench config (run on the GPU box from
# the repo root).  Each counter group is its own --pmc pass under its own kill
# timer (no trace domains in a PMC run):
#   fetch : FETCH_SIZE (HBM reads; x2 on gfx950, MI355X_MICROARCH.md §HBM)
#   sq    : LDS bank conflicts / LDS-active cycles, VALU + LDS instruction
#           counts, wave cycles, busy cycles
#   busy  : GRBM_GUI_ACTIVE (clock), VALU / LDS / any active-issue cycles,
#           LDS issue stalls, parked cycles
# then tools/prof_summary.py reduces them to profiles/<tag>/pmc_summary.json.
# Usage: bash tools/pmc.sh <tag> <config> [gb]
set -o pipefail
TAG=$1
CFG=${2:-2}
GB=${3:-}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--config $CFG --steps 1 --warmup 0 --no-cpu --no-parity"
[ -n "$GB" ] && ARGS="$ARGS --gb $GB"
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -f csv -d $OUT/$name -o run -- python3 bench.py $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; return 1; }
  echo "pass $name ok"
}
pass fetch FETCH_SIZE && \
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU && \
pass busy GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY
