#!/bin/bash
# r04aa: configs[3] with layers on two engines (analyze of layer k+1 overlaps layer k) + union allow-path DFA
set -o pipefail
mkdir -p gpurun_out/r04aa
export TMPDIR=/tmp
O=gpurun_out/r04aa
timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_analyzer.py tests/test_gpu_reentrancy.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TSG_C3_TRACE=1 timeout -k 10 400 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu > $O/c3.log 2> $O/c3.err || { echo "c3 failed"; tail -20 $O/c3.err; exit 1; }
tail -8 $O/c3.err
tail -1 $O/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['ms_per_step'], d['host_ms'], d['parity']['planted_found'], d['parity']['planted'], d['parity']['decoys_found'], d['parity']['spot_mismatched_files'])"
