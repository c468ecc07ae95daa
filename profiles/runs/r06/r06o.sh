set -o pipefail
bash tools/gpu_run.sh r06o trace4 c4 trace2 trace1 || exit 1
for c in 1 2 4; do python3 tools/timeline.py gpurun_out/r06o/trace_c$c/run_kernel_trace.csv > gpurun_out/r06o/timeline_c$c.txt; done
