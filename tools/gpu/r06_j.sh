#!/bin/bash
# r06 (j): A/B of the decision / outer-loop kernels' load batching (libtmpc_before.so = the previous
# build) on the streamed configs 3, 4 and the headline, then the stream / soft / iLQR / config / SQP tests
set -o pipefail
cd /root/repo
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 300 env TMPC_LIBRARY=$PWD/trajoptmpcreference_amd/libtmpc_before.so python -u tools/debug/r06_stream_probe.py c3:16:2 c4:16:2 head:8:1 > $O/probe_before.jsonl 2>&1 && \
timeout -k 10 300 python -u tools/debug/r06_stream_probe.py c3:16:2 c4:16:2 head:8:1 > $O/probe_after.jsonl 2>&1 && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_soft.py tests/test_gpu_ilqr.py tests/test_gpu_configs.py tests/test_gpu_sqp.py tests/test_gpu_hard.py -x -q --timeout 240 --timeout-method thread > $O/tests.txt 2>&1
