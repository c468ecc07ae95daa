set -o pipefail
BENCH_ARGS="--config 1" bash tools/ab_trace.sh r06zh_c1 "TSG_KW_DRAIN=64 TSG_KW_DRAIN=40 TSG_KW_DRAIN=32 TSG_KW_DRAIN=24 TSG_KW_DRAIN=48 TSG_KW_DRAIN=64 TSG_KW_DRAIN=32" || exit 1
