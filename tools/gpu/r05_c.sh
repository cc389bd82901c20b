# round 5 (c): neighbour-flag PCG (libtmpc_flags.so) vs full barriers (libtmpc_r05base.so): parity of the
# PCG paths on the flags build, then an A/B/A/B headline bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05c; mkdir -p $O
export TMPC_LIBRARY=/root/repo/trajoptmpcreference_amd/libtmpc_flags.so
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_pcg.py tests/test_gpu_sqp.py tests/test_gpu_long_horizon.py tests/test_gpu_plugins.py \
  tests/test_gpu_configs.py > $O/tests_flags.log 2>&1
echo "tests rc=$?" | tee $O/rc.txt
for v in r05base flags r05base flags; do
  TMPC_LIBRARY=/root/repo/trajoptmpcreference_amd/libtmpc_$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python -c "import json;d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['kernels']['qp']['avg_ms'])" | tee -a $O/ab.txt
done
