set -o pipefail
bash tools/gpu_run.sh r06t "pytest:analyzer or layer or stress or parity or shared" || exit 1
bash tools/ab_lib.sh r06t_ab "4 2" 2 "cur alt" || exit 1
