# round 5 (ad): config 3 forward sweep -- phase stamps (shipped order vs the next knot's prefetch issued
# after this knot's stores, TMPC_FWD_PF_LATE), config-3 bench both ways, iLQR parity with the variant
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05ad; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
for v in iS iPS; do
  TMPC_LIBRARY=$L/libtmpc_$v.so timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 \
    --solver ilqr --limits torque-al --no-cpu-baseline --no-secondary --no-hard-line > $O/stamps_c3_$v.out 2> $O/stamps_c3_$v.err || exit 1
  echo $v; grep ilqr_fwd $O/stamps_c3_$v.out | tail -2
done
for v in new iP; do
  lib=$L/libtmpc_$v.so; [ $v = new ] && lib=$L/libtmpc.so
  TMPC_LIBRARY=$lib timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline \
    --no-secondary --no-hard-line > $O/c3_$v.json 2> $O/c3_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1]);print('c3 $v', d['value'], {k: round(v['avg_ms'],4) for k, v in d['kernels'].items()})" | tee -a $O/summary.txt
done
TMPC_LIBRARY=$L/libtmpc_iP.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ilqr.py tests/test_gpu_configs.py -k "ilqr or config3" > $O/tests_iP.out 2>&1 || { echo tests failed; tail -30 $O/tests_iP.out; exit 1; }
echo tests ok; tail -1 $O/tests_iP.out
