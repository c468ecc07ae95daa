set -o pipefail
bash tools/gpu_run.sh r06z "pytest:gate or kw_states or stress" || exit 1
bash tools/ab_lib.sh r06z_ab "1" 3 "cur alt" || exit 1
