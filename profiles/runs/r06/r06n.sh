set -o pipefail
bash tools/gpu_run.sh r06n_c0 c0 || exit 1
BENCH_ARGS="--staged" bash tools/gpu_run.sh r06n_c0s c0 || exit 1
bash tools/gpu_run.sh r06n_c3 c3 || exit 1
BENCH_ARGS="--oracle-parity --no-cpu" bash tools/gpu_run.sh r06n_c2o c2 || exit 1
