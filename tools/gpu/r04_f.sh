# round 4 (f): the full-unroll build + register-slot hard PCG: full GPU suite, smoke, bench lines -> gpurun_out/r04f
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04f; mkdir -p $O
B=/root/repo/bench.py
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
prc=$?; echo "pytest rc=$prc" > $O/rc.txt
[ $prc -eq 0 ] || exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?" >> $O/rc.txt
run() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python $B "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc
}
run bench_hard_as 300 --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline && \
run bench_head 300 --steps 10 --warmup 2 --no-cpu-baseline && \
run bench_c3_fp32 300 --steps 3 --warmup 1 --solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline && \
run bench_c4 300 --steps 3 --warmup 1 --limits torque-joint-al --no-cpu-baseline
echo "all rc=$?" >> $O/rc.txt
exit 0
