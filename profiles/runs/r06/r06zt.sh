set -o pipefail
BENCH_ARGS="--oracle-parity --no-cpu" bash tools/gpu_run.sh r06zt c2full || exit 1
