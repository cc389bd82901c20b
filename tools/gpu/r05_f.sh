# round 5 (f): k_hard_pcg with address-space typed preconditioner reads (no flat loads) and the VALU
# butterfly (hA: typed reads only): hard parity, probe A/B, hard bench at B = 1024 / 4096; kernel-trace
# stats of the default bench (csv)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05f; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok
for v in hold hA new hC; do
  lib=$L/libtmpc_$v.so; [ $v = new ] && lib=$L/libtmpc.so
  TMPC_LIBRARY=$lib timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 1024 > $O/probe_$v.jsonl 2> $O/probe_$v.err || exit 1
  echo $v $(python -c "
import json
for l in open('$O/probe_$v.jsonl'):
    d=json.loads(l); k=list(d)[0]; print(k, round(d[k]['us_per_iteration'],3), round(d[k]['ms_iter0'],4), end=' ')") | tee -a $O/probe.txt
done
for b in 1024 4096; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
    --no-secondary > $O/hard_B$b.json 2> $O/hard_B$b.err || exit 1
  python -c "import json;d=json.loads(open('$O/hard_B$b.json').read().strip().splitlines()[-1]);print('hard B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'])" | tee -a $O/probe.txt
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default -o run -- python3 /root/repo/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_default.out 2>&1) || exit 1
echo prof done
