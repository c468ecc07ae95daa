set -o pipefail
bash tools/gpu_run.sh r06zr pytest || exit 1
bash tools/ab_lib.sh r06zr_ab "2 1" 3 "cur alt" || exit 1
