# round 5 (n/o): k_hard_pcg setup restructured (GJ rows in registers, stairs staged cooperatively in LDS):
# (stair, column) without LDS staging): hard / pendulum / banded-SQP / dense parity, probe, setup + phase
# stamps, hard bench B = 4096; the hard line's mismatch probe with the line-search replay
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05o; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py tests/test_gpu_long_horizon.py tests/test_gpu_pcg_dense.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok
timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 1024 > $O/probe.jsonl 2> $O/probe.err || exit 1
python -c "
import json
for l in open('$O/probe.jsonl'):
    d=json.loads(l); k=list(d)[0]; print('new', k, round(d[k]['us_per_iteration'],3), round(d[k]['ms_iter0'],4), round(d[k]['ms_iter100'],4))" | tee -a $O/probe.txt
TMPC_LIBRARY=$L/libtmpc_hS.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_hS.txt 2> $O/probe_hS.err || exit 1
grep hx_setup $O/probe_hS.txt | head -3
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch 4096 --limits torque-velocity-as --no-cpu-baseline \
  --no-secondary > $O/hard_B4096.json 2> $O/hard_B4096.err || exit 1
python -c "import json;d=json.loads(open('$O/hard_B4096.json').read().strip().splitlines()[-1]);print('hard B4096', d['value'], d['kernels']['hard_pcg']['avg_ms'], d['kernels']['hard_schur']['avg_ms'])" | tee -a $O/probe.txt
timeout -k 10 300 python -u tools/debug/r05_hard_mismatch.py 5 > $O/mismatch.jsonl 2> $O/mismatch.err || { tail -20 $O/mismatch.err; exit 1; }
echo mismatch done
