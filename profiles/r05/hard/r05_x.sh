# round 5 (x): k_hard_schur phase 2: unit pieces read one Y entry (uv y_uc + 0), not the full product
# hard / pendulum / banded-SQP parity, setup stamps, probe, hard bench B = 1024 / 4096
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05x; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py tests/test_gpu_long_horizon.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok; tail -1 $O/tests.out
TMPC_LIBRARY=$L/libtmpc_hS.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_hS.txt 2> $O/probe_hS.err || exit 1
grep -h "hx_setup\|hs_stamps" $O/probe_hS.txt | head -8
timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 1024 > $O/probe.jsonl 2> $O/probe.err || exit 1
python -c "
import json
for l in open('$O/probe.jsonl'):
    d=json.loads(l); k=list(d)[0]; print('new', k, round(d[k]['us_per_iteration'],3), round(d[k]['ms_iter0'],4), round(d[k]['ms_iter100'],4))" | tee -a $O/probe.txt
for b in 1024 4096; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
    --no-secondary > $O/hard_B$b.json 2> $O/hard_B$b.err || exit 1
  python -c "import json;d=json.loads(open('$O/hard_B$b.json').read().strip().splitlines()[-1]);print('hard B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'], d['kernels']['hard_schur']['avg_ms'])" | tee -a $O/probe.txt
done
