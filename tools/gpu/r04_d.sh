# round 4 (d): iLQR replay tests -> gpurun_out/r04d
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ilqr.py tests/test_gpu_mpc.py tests/test_gpu_configs.py -v -rA --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?" > $O/rc.txt
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err; echo "bench rc=$?" >> $O/rc.txt
exit 0
