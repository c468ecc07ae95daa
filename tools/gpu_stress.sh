set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stress.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_stress.log 2>&1 || { echo "stress tests failed"; tail -40 gpurun_out/pytest_stress.log; exit 1; }
tail -5 gpurun_out/pytest_stress.log
timeout -k 10 300 python -u bench.py --config 1 --no-parity > gpurun_out/bench_c1.log 2>&1 || { echo c1 failed; tail -20 gpurun_out/bench_c1.log; exit 1; }
tail -1 gpurun_out/bench_c1.log
timeout -k 10 400 python -u bench.py --config 4 --gb 10 --steps 2 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || { echo c4 failed; tail -20 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log
