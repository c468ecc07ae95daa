set -o pipefail
bash tools/gpu_run.sh r06u trace4 || exit 1
python3 tools/timeline.py gpurun_out/r06u/trace_c4/run_kernel_trace.csv > gpurun_out/r06u/timeline_c4.txt
