# round 5 (ai): iLQR backward sweep -- the prefetched A_{k-1}, B_{k-1} written to LDS before the knot's
# K / d stores (iK: TMPC_BWD_AB_EARLY); stamps (iS0 shipped, iKS), config-3 and iLQR bench, iLQR parity
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05ai; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
for v in iS0 iKS; do
  TMPC_LIBRARY=$L/libtmpc_$v.so timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 \
    --solver ilqr --limits torque-al --no-cpu-baseline --no-secondary --no-hard-line > $O/stamps_c3_$v.out 2> $O/stamps_c3_$v.err || exit 1
  echo $v; grep ilqr_stamps $O/stamps_c3_$v.out | tail -n 2
done
for v in new iK; do
  lib=$L/libtmpc_$v.so; [ $v = new ] && lib=$L/libtmpc.so
  for cfg in c3 ilqr; do
    args="--solver ilqr --no-cpu-baseline --no-secondary --no-hard-line"
    [ $cfg = c3 ] && args="$args --limits torque-al --steps 2 --warmup 1" || args="$args --steps 5 --warmup 2"
    TMPC_LIBRARY=$lib timeout -k 10 300 python3 bench.py $args > $O/${cfg}_$v.json 2> $O/${cfg}_$v.err || exit 1
    python3 -c "import json;d=json.loads(open('$O/${cfg}_$v.json').read().strip().splitlines()[-1]);print('$cfg $v', d['value'], {k: round(v['avg_ms'],4) for k, v in d['kernels'].items() if k.startswith('ilqr')})" | tee -a $O/summary.txt
  done
done
TMPC_LIBRARY=$L/libtmpc_iK.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ilqr.py tests/test_gpu_configs.py tests/test_gpu_precision.py -k "ilqr or config3 or config5" > $O/tests_iK.out 2>&1 || { echo tests iK failed; tail -30 $O/tests_iK.out; exit 1; }
echo tests iK ok; tail -n 1 $O/tests_iK.out
