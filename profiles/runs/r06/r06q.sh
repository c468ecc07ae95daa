set -o pipefail
bash tools/gpu_run.sh r06q "pytest:small_sort or analyzer or parity or stress or exclude or dense" || exit 1
bash tools/ab_lib.sh r06q_ab "2" 3 "cur alt" || exit 1
