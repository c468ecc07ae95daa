set -o pipefail
bash tools/gpu_run.sh r06m "pytest:kw_states or gate" || exit 1
bash tools/ab_lib.sh r06m_ab "1" 2 "cur alt" || exit 1
