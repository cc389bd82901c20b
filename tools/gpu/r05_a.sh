# round 5 (a): the exact-replay parity tests (canonical order for both lane layouts, GM + warm start,
# pendulum hard replay, PCG-J order-decided QPs)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sqp.py tests/test_gpu_long_horizon.py tests/test_gpu_pendulum.py tests/test_gpu_pcg.py \
  > $O/tests.log 2>&1
echo "tests rc=$?" | tee $O/rc.txt
tail -30 $O/tests.log
