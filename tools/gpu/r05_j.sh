# round 5 (j): k_hard_pcg with the first streamed batch in flight during the register-held products
# (U = 8 shipped, U = 12 variant): hard parity, probe A/B (r04 library, r05i build, new, U = 12), phase
# stamps, hard bench; config-4 PMC FETCH / WRITE passes on the r05 library (the secondary's traffic)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05j; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok
for v in hold hI new hF12; do
  lib=$L/libtmpc_$v.so; [ $v = new ] && lib=$L/libtmpc.so
  TMPC_LIBRARY=$lib timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 1024 > $O/probe_$v.jsonl 2> $O/probe_$v.err || exit 1
  python -c "
import json
for l in open('$O/probe_$v.jsonl'):
    d=json.loads(l); k=list(d)[0]; print('$v', k, round(d[k]['us_per_iteration'],3), round(d[k]['ms_iter0'],4))" | tee -a $O/probe.txt
done
TMPC_LIBRARY=$L/libtmpc_hS8.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_hS8.txt 2> $O/probe_hS8.err || exit 1
for b in 1024 4096; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
    --no-secondary > $O/hard_B$b.json 2> $O/hard_B$b.err || exit 1
  python -c "import json;d=json.loads(open('$O/hard_B$b.json').read().strip().splitlines()[-1]);print('hard B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'], d['kernels']['hard_schur']['avg_ms'])" | tee -a $O/probe.txt
done
B=/root/repo/bench.py
C4="--limits torque-joint-al --steps 1 --warmup 1 --no-cpu-baseline --no-secondary"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c4 -o run -- python3 $B $C4 > $O/fetch_c4.out 2>&1) || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c4 -o run -- python3 $B $C4 > $O/write_c4.out 2>&1) || exit 1
echo pmc done
