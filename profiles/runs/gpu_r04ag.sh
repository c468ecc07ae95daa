#!/bin/bash
# r04ag: lazy newline edge-case GPU tests
set -o pipefail
mkdir -p gpurun_out/r04ag
export TMPDIR=/tmp
O=gpurun_out/r04ag
timeout -k 10 600 python -u -m pytest tests/test_gpu_lazy_lines.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
