# round 5 (y): k_hard_schur phase 2 -- unit pieces of either side read one Y entry (a -[A B] row against a
# unit column reads its own Y), only the -[A B] x -[A B] entries take the full product; shipped (EPS 2)
# vs EPS 1; hard / pendulum / banded-SQP parity, schur stamps, hard bench B = 1024 / 4096
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05y; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py tests/test_gpu_long_horizon.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok; tail -1 $O/tests.out
TMPC_LIBRARY=$L/libtmpc_hS.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_hS.txt 2> $O/probe_hS.err || exit 1
grep -h "hs_stamps" $O/probe_hS.txt | head -4
for v in new hE1; do
  lib=$L/libtmpc_$v.so; [ $v = new ] && lib=$L/libtmpc.so
  for b in 1024 4096; do
    TMPC_LIBRARY=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
      --no-secondary > $O/hard_${v}_B$b.json 2> $O/hard_${v}_B$b.err || exit 1
    python -c "import json;d=json.loads(open('$O/hard_${v}_B$b.json').read().strip().splitlines()[-1]);print('hard $v B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'], d['kernels']['hard_schur']['avg_ms'], d['hard_limits']['parity'] if 'hard_limits' in d else '')" | tee -a $O/probe.txt
  done
done
