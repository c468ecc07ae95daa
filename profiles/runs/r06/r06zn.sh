set -o pipefail
TSG_LIB_VARIANT=exp TSG_SCAN_MODE=8 bash tools/pmc.sh r06zn_tri 2 || exit 1
TSG_LIB_VARIANT=exp bash tools/pmc.sh r06zn_exp 2 || exit 1
