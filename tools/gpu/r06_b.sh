#!/bin/bash
# r06: stream hand-over folded into k_soft_outer, activation in the INIT decisions; parity + rates
set -o pipefail
mkdir -p gpurun_out/r06b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_soft.py tests/test_gpu_configs.py tests/test_gpu_ilqr.py tests/test_gpu_mpc.py tests/test_gpu_pendulum.py > gpurun_out/r06b/tests.txt 2>&1 || { tail -30 gpurun_out/r06b/tests.txt; exit 1; }
tail -3 gpurun_out/r06b/tests.txt
timeout -k 10 400 python -u tools/debug/r06_stream_probe.py head c4 hard c3 c2 > gpurun_out/r06b/probe.jsonl 2>&1 || { tail -30 gpurun_out/r06b/probe.jsonl; exit 1; }
cat gpurun_out/r06b/probe.jsonl
