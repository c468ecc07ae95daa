set -o pipefail
bash tools/gpu_run.sh r06e "pytest:kw_states or gate or parity or stress" || exit 1
bash tools/gpu_run.sh r06e pytest trace2 trace1 c2 c1 || exit 1
for c in 1 2; do python3 tools/timeline.py gpurun_out/r06e/trace_c$c/run_kernel_trace.csv > gpurun_out/r06e/timeline_c$c.txt; done
grep -E "k_scan_fast|k_report|k_path_gate|k_region" gpurun_out/r06e/timeline_c2.txt | tail -4
