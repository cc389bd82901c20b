# round 5 (ae): config 3 forward sweep -- phase stamps and bench: shipped; the next knot's prefetch issued
# after this knot's stores (iP: TMPC_FWD_PF_LATE); explicit vmcnt(0) after the loads into xh / uh so the
# compiler's wait pass puts no full wait inside the knot loop (iW: TMPC_FWD_WAITS); iLQR parity with both
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05ae; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
for v in iS iPS iWS; do
  TMPC_LIBRARY=$L/libtmpc_$v.so timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 \
    --solver ilqr --limits torque-al --no-cpu-baseline --no-secondary --no-hard-line > $O/stamps_c3_$v.out 2> $O/stamps_c3_$v.err || exit 1
  echo $v; grep ilqr_fwd $O/stamps_c3_$v.out | tail -n 2
done
for v in new iP iW; do
  lib=$L/libtmpc_$v.so; [ $v = new ] && lib=$L/libtmpc.so
  TMPC_LIBRARY=$lib timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline \
    --no-secondary --no-hard-line > $O/c3_$v.json 2> $O/c3_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1]);print('c3 $v', d['value'], {k: round(v['avg_ms'],4) for k, v in d['kernels'].items()})" | tee -a $O/summary.txt
done
for v in iP iW; do
  TMPC_LIBRARY=$L/libtmpc_$v.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_ilqr.py tests/test_gpu_configs.py -k "ilqr or config3" > $O/tests_$v.out 2>&1 || { echo tests $v failed; tail -30 $O/tests_$v.out; exit 1; }
  echo tests $v ok; tail -n 1 $O/tests_$v.out
done
