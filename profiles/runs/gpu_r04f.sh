#!/bin/bash
# r04f: forced-split parity tests, GPU suite, configs[2] / configs[4] lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify_split.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r04f_split.log 2>&1 || { echo "split tests failed"; tail -40 gpurun_out/pytest_r04f_split.log; exit 1; }
tail -2 gpurun_out/pytest_r04f_split.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r04f.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r04f.log; exit 1; }
tail -2 gpurun_out/pytest_r04f.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_c2_r04f.log 2>&1 || { echo "bench c2 failed"; tail -20 gpurun_out/bench_c2_r04f.log; exit 1; }
tail -1 gpurun_out/bench_c2_r04f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'], d['stages_ms'], d['counts'], d['parity']['spot_mismatched_files'], d['parity']['planted_found'], d['parity']['decoys_found'], d['cpu_baseline']['value'])"
timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c4_r04f.log 2>&1 || { echo "bench c4 failed"; tail -20 gpurun_out/bench_c4_r04f.log; exit 1; }
tail -1 gpurun_out/bench_c4_r04f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms'], d['counts'], d['parity']['stress_mismatched_files'], d['parity']['spot_mismatched_files'])"
