# round 5 (b): replay / plugin / boundary / hard parity tests, then a headline bench (structural A/B reads)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05b; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_plugins.py tests/test_gpu_sqp.py tests/test_gpu_long_horizon.py tests/test_gpu_pendulum.py \
  tests/test_gpu_pcg.py tests/test_gpu_boundary.py tests/test_gpu_hard.py > $O/tests.log 2>&1
echo "tests rc=$?" | tee $O/rc.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err
echo "bench rc=$?" | tee -a $O/rc.txt
tail -c 1500 $O/bench.json
