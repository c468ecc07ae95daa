set -o pipefail
bash tools/gpu_run.sh r06v "pytest:verify_split or stress or empty_match or big or custom or allow" || exit 1
bash tools/ab_lib.sh r06v_ab "4" 2 "cur alt" || exit 1
