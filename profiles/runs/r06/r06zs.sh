set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06zs
mkdir -p $O
bash tools/gpu_run.sh r06zs smoke || exit 1
# the driver's own command (defaults: configs[2], cpu_baseline, parity)
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -n 1 $O/bench_default.log | cut -c1-400
# the same command under rocprofv3: the bench line's avg_launch_ms and the kernel stats from one run
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_default -o run -- python3 bench.py > $O/trace_default.log 2>&1 || { echo "trace failed"; tail -20 $O/trace_default.log; exit 1; }
python3 tools/timeline.py $O/trace_default/run_kernel_trace.csv > $O/timeline_default.txt
bash tools/gpu_run.sh r06zs c1 c4 || exit 1
