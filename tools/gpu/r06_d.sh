#!/bin/bash
# r06: arm6 hard-limit parity (oracle fixture, in-test classification), pivoting plugin QP, LDS bound
set -o pipefail
mkdir -p gpurun_out/r06d
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -rw --timeout 300 --timeout-method thread tests/test_gpu_hard_arm6.py tests/test_gpu_plugins.py tests/test_gpu_long_horizon.py tests/test_gpu_stream.py > gpurun_out/r06d/tests.txt 2>&1 || { tail -40 gpurun_out/r06d/tests.txt; exit 1; }
tail -25 gpurun_out/r06d/tests.txt
