# round 5 (i): k_hard_pcg products without selects (zero band past each row, zeroed register entries, p
# guard): hard / pendulum / banded-SQP parity on the shipped build (REG 24), probe A/B against REG 20 / 16
# and the r04 library, phase stamps, hard bench B = 1024 / 4096
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05i; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py tests/test_gpu_long_horizon.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok
for v in hold new hE20 hE16; do
  lib=$L/libtmpc_$v.so; [ $v = new ] && lib=$L/libtmpc.so
  TMPC_LIBRARY=$lib timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 1024 > $O/probe_$v.jsonl 2> $O/probe_$v.err || exit 1
  python -c "
import json
for l in open('$O/probe_$v.jsonl'):
    d=json.loads(l); k=list(d)[0]; print('$v', k, round(d[k]['us_per_iteration'],3), round(d[k]['ms_iter0'],4))" | tee -a $O/probe.txt
done
TMPC_LIBRARY=$L/libtmpc_hS24.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_hS24.txt 2> $O/probe_hS24.err || exit 1
for b in 1024 4096; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
    --no-secondary > $O/hard_B$b.json 2> $O/hard_B$b.err || exit 1
  python -c "import json;d=json.loads(open('$O/hard_B$b.json').read().strip().splitlines()[-1]);print('hard B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'], d['kernels']['hard_schur']['avg_ms'])" | tee -a $O/probe.txt
done
