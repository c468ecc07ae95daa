set -o pipefail
bash tools/gpu_run.sh r06b pytest || exit 1
BENCH_ARGS="" bash tools/ab_trace.sh r06b_ab "TSG_VERIFY_NARROW=1 - TSG_VERIFY_JPW=8 TSG_VERIFY_JPW=32" > gpurun_out/r06b_ab.txt 2>&1 || { tail -5 gpurun_out/r06b_ab.txt; exit 1; }
cat gpurun_out/r06b_ab.txt
bash tools/gpu_run.sh r06b c2
