#!/bin/bash
# r03g: the other BASELINE configs on the current tree: configs[0] (host batch,
# PCIe-inclusive), configs[1] (prefilter only), configs[3] (layer tars) and its
# shared-list mode.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 1 0 3; do
  timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 > gpurun_out/bench_c${c}_r03g.log 2>&1 || { echo "bench c$c failed"; tail -20 gpurun_out/bench_c${c}_r03g.log; exit 1; }
  tail -1 gpurun_out/bench_c${c}_r03g.log | cut -c1-1500
done
timeout -k 10 400 python -u bench.py --config 3 --shared --steps 5 --warmup 2 > gpurun_out/bench_c3s_r03g.log 2>&1 || { echo "bench c3 shared failed"; tail -20 gpurun_out/bench_c3s_r03g.log; exit 1; }
tail -1 gpurun_out/bench_c3s_r03g.log | cut -c1-1500
