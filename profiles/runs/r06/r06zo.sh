set -o pipefail
bash tools/gpu_run.sh r06zo "pytest:parity or kw_states or gate" || exit 1
bash tools/ab_lib.sh r06zo_ab "2 1" 3 "cur alt" || exit 1
