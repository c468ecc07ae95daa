set -o pipefail
bash tools/gpu_run.sh r06f "pytest:kw_states or gate" || exit 1
BENCH_ARGS="--config 1" bash tools/ab_trace.sh r06f_c1 "TSG_KW_DRAIN=0 - TSG_KW_DRAIN=8 TSG_KW_DRAIN=32" || exit 1
bash tools/ab_trace.sh r06f_c2 "TSG_KW_DRAIN=0 - TSG_KW_DRAIN=8 TSG_KW_DRAIN=32" || exit 1
