# round 4 (c): the integer-exactness rework (canonical PCG replay, single iLQR restatement + replay, config 3
# fp32 bounds) and the boundary tests -> gpurun_out/r04c
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_pcg.py tests/test_gpu_sqp.py tests/test_gpu_ilqr.py tests/test_gpu_configs.py tests/test_gpu_mpc.py tests/test_gpu_precision.py tests/test_gpu_boundary.py -v -rA --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?" > $O/rc.txt
exit 0
