set -o pipefail
bash tools/ab_trace.sh r06x_c2 "- TSG_KW_OFF=1 - TSG_KW_OFF=1" || exit 1
