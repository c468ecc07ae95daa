#!/bin/bash
# r04ak: product-library check after the k_nl_spans loop (lazy-line, parity, split tests) + byte-range split of one
# 20 GB file into 2 / 4 / 8 parts (tools/split_bench.py)
set -o pipefail
mkdir -p gpurun_out/r04ak
export TMPDIR=/tmp
O=gpurun_out/r04ak
timeout -k 10 600 python -u -m pytest tests/test_gpu_lazy_lines.py tests/test_gpu_parity.py tests/test_split.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python -u tools/split_bench.py --gb 20 --parts 2 4 8 --reps 3 > $O/split_bench.log 2>&1 || { echo "split bench failed"; tail -20 $O/split_bench.log; exit 1; }
tail -1 $O/split_bench.log | cut -c1-1500
