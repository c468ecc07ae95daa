set -o pipefail
bash tools/gpu_run.sh r06c pytest || exit 1
bash tools/ab_trace.sh r06c_ab "- TSG_VERIFY_SPLIT=1 TSG_VERIFY_JPW=64 TSG_NL_EARLY=1" > gpurun_out/r06c_ab.txt 2>&1 || { tail -5 gpurun_out/r06c_ab.txt; exit 1; }
cat gpurun_out/r06c_ab.txt
bash tools/gpu_run.sh r06c c2 c4
