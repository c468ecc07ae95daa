set -o pipefail
bash tools/gpu_run.sh r06i trace2 trace1 c2 c1 || exit 1
for c in 1 2; do python3 tools/timeline.py gpurun_out/r06i/trace_c$c/run_kernel_trace.csv > gpurun_out/r06i/timeline_c$c.txt; done
grep -E "k_scan_fast|k_report|span" gpurun_out/r06i/timeline_c2.txt | tail -3
grep -E "k_scan_fast|k_report|span" gpurun_out/r06i/timeline_c1.txt | tail -3
