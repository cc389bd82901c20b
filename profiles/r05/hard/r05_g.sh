# round 5 (g): k_hard_pcg phase stamps (timing build hS) on the probe; the C build (slot-0 z / S p in
# registers, setup staged in the cache tail) on the hard parity suite, probe and hard bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05g; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
TMPC_LIBRARY=$L/libtmpc_hS.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_hS.txt 2> $O/probe_hS.err || exit 1
echo stamps done
TMPC_LIBRARY=$L/libtmpc_hC.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py > $O/tests_hC.out 2>&1 || { echo tests failed; tail -30 $O/tests_hC.out; exit 1; }
echo tests ok
TMPC_LIBRARY=$L/libtmpc_hC.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 1024 > $O/probe_hC.jsonl 2> $O/probe_hC.err || exit 1
python -c "
import json
for l in open('$O/probe_hC.jsonl'):
    d=json.loads(l); k=list(d)[0]; print('hC', k, round(d[k]['us_per_iteration'],3), round(d[k]['ms_iter0'],4))" | tee -a $O/probe.txt
for b in 1024 4096; do
  TMPC_LIBRARY=$L/libtmpc_hC.so timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
    --no-secondary > $O/hard_B$b.json 2> $O/hard_B$b.err || exit 1
  python -c "import json;d=json.loads(open('$O/hard_B$b.json').read().strip().splitlines()[-1]);print('hard hC B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'])" | tee -a $O/probe.txt
done
