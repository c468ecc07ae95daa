set -o pipefail
bash tools/gpu_run.sh r06h "pytest:kw_states or gate or parity or stress" || exit 1
BENCH_ARGS="--config 1" bash tools/ab_trace.sh r06h_c1 "TSG_KW_DRAIN=0 - TSG_KW_DRAIN=40 TSG_KW_DRAIN=80" || exit 1
bash tools/ab_trace.sh r06h_c2 "TSG_KW_DRAIN=0 - TSG_KW_DRAIN=40 TSG_KW_DRAIN=80" || exit 1
