#!/bin/bash
# r06 (k): fp32 Riccati on the matrix cores (k_ilqr_backward<NJ, float, true>) against the fp32 VALU sweep:
# config 3 fp32 accuracy vs the fp64 oracle (8 problems) and the streamed config-3 fp32 line, both instances
set -o pipefail
cd /root/repo
O=gpurun_out/r06k; mkdir -p $O
B="python -u bench.py --solver ilqr --limits torque-al --precision fp32 --substreams 2 --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --lockstep-steps 0"
timeout -k 10 240 python -u tools/debug/r06_fp32_probe.py > $O/fp32_probe_mf.txt 2>&1 && \
timeout -k 10 240 env TMPC_ILQR_F32_VALU=1 python -u tools/debug/r06_fp32_probe.py > $O/fp32_probe_valu.txt 2>&1 && \
timeout -k 10 300 $B > $O/bench_c3f32_mf.json 2> $O/bench_c3f32_mf.err && \
timeout -k 10 300 env TMPC_ILQR_F32_VALU=1 $B > $O/bench_c3f32_valu.json 2> $O/bench_c3f32_valu.err && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_ilqr.py tests/test_gpu_configs.py -q --timeout 240 --timeout-method thread > $O/tests.txt 2>&1
