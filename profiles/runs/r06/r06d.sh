set -o pipefail
bash tools/gpu_run.sh r06d pytest trace2 c2 || exit 1
python3 tools/timeline.py gpurun_out/r06d/trace_c2/run_kernel_trace.csv > gpurun_out/r06d/timeline_c2.txt
head -14 gpurun_out/r06d/timeline_c2.txt
