# round 5 (s): k_hard_schur with 4 S entries per step (NJ <= 6) and no HBM copies of the LDS-cached
# preconditioner blocks: hard parity, hard bench (shipped vs EPS = 2), default bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05s; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py tests/test_gpu_long_horizon.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok
for v in new hE2; do
  lib=$L/libtmpc_$v.so; [ $v = new ] && lib=$L/libtmpc.so
  for b in 1024 4096; do
    TMPC_LIBRARY=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
      --no-secondary > $O/hard_${v}_B$b.json 2> $O/hard_${v}_B$b.err || exit 1
    python -c "import json;d=json.loads(open('$O/hard_${v}_B$b.json').read().strip().splitlines()[-1]);print('hard $v B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'], d['kernels']['hard_schur']['avg_ms'])" | tee -a $O/probe.txt
  done
done
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo "default rc=$?"
