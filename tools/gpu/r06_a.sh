#!/bin/bash
# r06: continuous-batching parity (stream == batch bitwise) and the first stream-vs-lockstep rates
set -o pipefail
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream.py > gpurun_out/r06a/tests_stream.txt 2>&1 || { tail -30 gpurun_out/r06a/tests_stream.txt; exit 1; }
tail -3 gpurun_out/r06a/tests_stream.txt
timeout -k 10 400 python -u tools/debug/r06_stream_probe.py head c4 hard c3 c2 > gpurun_out/r06a/probe.jsonl 2>&1 || { tail -30 gpurun_out/r06a/probe.jsonl; exit 1; }
cat gpurun_out/r06a/probe.jsonl
