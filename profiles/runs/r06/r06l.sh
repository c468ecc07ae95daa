set -o pipefail
bash tools/gpu_run.sh r06l "pytest:kw_states or gate or parity or stress" || exit 1
bash tools/ab_lib.sh r06l_ab "2 1" 2 "cur alt" || exit 1
