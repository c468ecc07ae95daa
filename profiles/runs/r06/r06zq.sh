set -o pipefail
bash tools/ab_trace.sh r06zq_c2 "- TSG_NOCOUNT=1 - TSG_NOCOUNT=1 - TSG_NOCOUNT=1" || exit 1
