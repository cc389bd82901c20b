# round 3 (session 2): V_xx symmetrisation folded into the next knot fragment build: GPU suite + config 3 / 5 iLQR lines + config 3 trace, PMC
# summaries of profiles/pmc (r03/v5) in place, plus smoke() -> gpurun_out/r03w
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r03w; mkdir -p $O
B=/root/repo/bench.py
run() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python $B "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc
}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
prc=$?; echo "pytest rc=$prc" > $O/rc.txt
[ $prc -eq 0 ] || exit 0
run bench_c3_fp64 300 --steps 3 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline && \
run bench_c5_ilqr 300 --steps 3 --warmup 1 --N 128 --solver ilqr --batch 8192 --mpc-steps 4 --no-cpu-baseline && \
run bench_c3_fp32 300 --steps 3 --warmup 1 --solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 $B --steps 1 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline > $O/trace_c3.out 2>&1); echo "trace_c3 rc=$?" >> $O/rc.txt
echo "all rc=$?" >> $O/rc.txt
exit 0
