set -o pipefail
bash tools/gpu_run.sh r06p "pytest:small_sort" || exit 1
bash tools/gpu_run.sh r06p pytest || exit 1
bash tools/ab_lib.sh r06p_ab "2 1" 2 "cur alt" || exit 1
