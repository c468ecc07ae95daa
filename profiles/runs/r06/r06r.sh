set -o pipefail
bash tools/gpu_run.sh r06r "pytest:small_sort" || exit 1
bash tools/ab_lib.sh r06r_ab "2" 2 "cur alt" || exit 1
bash tools/gpu_run.sh r06r trace2 || exit 1
python3 tools/timeline.py gpurun_out/r06r/trace_c2/run_kernel_trace.csv > gpurun_out/r06r/timeline_c2.txt
grep -E "k_tile|k_mark_jobs|k_loc_keys" gpurun_out/r06r/timeline_c2.txt | tail -12
