# round 5 (h): k_hard_pcg with branch-free S p, swizzled row-major LDS preconditioner blocks, unrolled
# fan-in, register band of 24 / 20 / 16 entries (hD24 / hD20 / hD16): hard parity on hD16, probe A/B,
# phase stamps (hS16), hard bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05h; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
TMPC_TEST_HARD_REG=16 TMPC_LIBRARY=$L/libtmpc_hD16.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py > $O/tests_hD16.out 2>&1 || { echo tests failed; tail -30 $O/tests_hD16.out; exit 1; }
echo tests ok
for v in hold hD24 hD20 hD16; do
  TMPC_LIBRARY=$L/libtmpc_$v.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 1024 > $O/probe_$v.jsonl 2> $O/probe_$v.err || exit 1
  python -c "
import json
for l in open('$O/probe_$v.jsonl'):
    d=json.loads(l); k=list(d)[0]; print('$v', k, round(d[k]['us_per_iteration'],3), round(d[k]['ms_iter0'],4))" | tee -a $O/probe.txt
done
TMPC_LIBRARY=$L/libtmpc_hS16.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_hS16.txt 2> $O/probe_hS16.err || exit 1
for v in hD24 hD16; do
for b in 1024 4096; do
  TMPC_LIBRARY=$L/libtmpc_$v.so timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
    --no-secondary > $O/hard_${v}_B$b.json 2> $O/hard_${v}_B$b.err || exit 1
  python -c "import json;d=json.loads(open('$O/hard_${v}_B$b.json').read().strip().splitlines()[-1]);print('hard $v B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'])" | tee -a $O/probe.txt
done
done
