#!/bin/bash
# Builds trivy_amd/libtrivy_secret_gpu_<name>.so (name alt, alt2, ...) from a
# revision's engine sources -- a git rev, or "WT" for the working tree --
# optionally with a patch applied on top, for same-box A/B runs against the
# working tree's library (TSG_LIB_VARIANT=<name>; tools/ab_lib.sh).
# Usage: bash tools/build_alt.sh <rev|WT> [patch] [name]
set -e
REV=$1; PATCH=$2; NAME=${3:-alt}
rm -rf build_$NAME && mkdir -p build_$NAME/src
if [ "$REV" = WT ]; then
  tar -c trivy_amd/csrc include | tar -x -C build_$NAME/src
else
  git archive "$REV" trivy_amd/csrc include | tar -x -C build_$NAME/src
fi
[ -n "$PATCH" ] && (cd build_$NAME/src && patch -p1 < "$PATCH")
make -j8 alt ALT=$NAME
