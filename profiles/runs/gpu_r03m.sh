#!/bin/bash
# r03m: the stress gate test alone, breadth-first numbering (exp build) then
# the product's frequency order, each with its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TSG_LIB_VARIANT=exp TSG_BIG_BFS=1 timeout -k 10 240 python -u -m pytest tests/test_gpu_stress.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_r03m_bfs.log 2>&1 || { echo "bfs run failed"; tail -60 gpurun_out/pytest_r03m_bfs.log; exit 1; }
tail -3 gpurun_out/pytest_r03m_bfs.log
timeout -k 10 240 python -u -m pytest tests/test_gpu_stress.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_r03m.log 2>&1 || { echo "product run failed"; tail -60 gpurun_out/pytest_r03m.log; exit 1; }
tail -3 gpurun_out/pytest_r03m.log
