# round 5 (q): k_hard_schur with the rows' piece knots and the shared Ghat in LDS: hard parity suite, schur
# phase stamps, hard bench B = 1024 / 4096
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05q; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py tests/test_gpu_long_horizon.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok
TMPC_LIBRARY=$L/libtmpc_hS.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 1024 \
  --limits torque-velocity-as --no-cpu-baseline --no-secondary > $O/schur_stamps.txt 2> $O/schur_stamps.err || exit 1
grep hs_stamps $O/schur_stamps.txt | head -4
for b in 1024 4096; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
    --no-secondary > $O/hard_B$b.json 2> $O/hard_B$b.err || exit 1
  python -c "import json;d=json.loads(open('$O/hard_B$b.json').read().strip().splitlines()[-1]);print('hard B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'], d['kernels']['hard_schur']['avg_ms'])" | tee -a $O/probe.txt
done
