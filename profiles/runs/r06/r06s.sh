set -o pipefail
bash tools/gpu_run.sh r06s pytest || exit 1
bash tools/ab_lib.sh r06s_ab "2 4" 2 "cur alt" || exit 1
