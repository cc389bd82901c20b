# round 5 (al): iLQR backward with branch-free MFMA fragment loads (libtmpc_iX.so = the shipped library
# with only tmpc_ilqr.hip's change): iLQR parity, iLQR / config-3 / config-5 lines, then the full suite,
# smoke and the default bench on it
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05al; mkdir -p $O
export TMPC_LIBRARY=/root/repo/trajoptmpcreference_amd/libtmpc_iX.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ilqr.py tests/test_gpu_configs.py tests/test_gpu_precision.py -k "ilqr or config3 or config5" > $O/tests_ilqr.out 2>&1 || { echo ilqr tests failed; tail -30 $O/tests_ilqr.out; exit 1; }
echo ilqr tests ok; tail -n 1 $O/tests_ilqr.out
B=/root/repo/bench.py
run() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u $B "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc" | tee -a $O/rc.txt; return $rc
}
run bench_c3 300 --steps 2 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline && \
run bench_ilqr 200 --steps 5 --warmup 2 --solver ilqr --no-cpu-baseline && \
run bench_c3_fp32 300 --steps 2 --warmup 1 --solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline && \
run bench_c5_ilqr 300 --steps 2 --warmup 1 --N 128 --batch 8192 --mpc-steps 4 --solver ilqr --no-cpu-baseline || exit 1
for n in bench_c3 bench_ilqr bench_c3_fp32 bench_c5_ilqr; do
  python3 -c "import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);print('$n', round(d['value'],1), {k: round(v['avg_ms'],4) for k, v in d['kernels'].items() if k.startswith('ilqr_')})"
done
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.out 2>&1
echo "tests rc=$?"; tail -n 1 $O/tests.out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.out 2>&1 || { echo smoke failed; tail $O/smoke.out; exit 1; }
echo smoke ok
run bench_default 900
python3 -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);print('default', round(d['value'],1), d['parity']['mismatches'], 'hard', round(d['hard_limits']['value'],1), 'c4', round(d['secondary']['value'],1))"
