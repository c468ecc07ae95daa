set -o pipefail
bash tools/gpu_run.sh r06y "pytest:verify or stress or parity or exclude or captures or group" || exit 1
bash tools/ab_lib.sh r06y_ab "2 4" 2 "cur alt" || exit 1
