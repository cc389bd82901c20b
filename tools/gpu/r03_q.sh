# round 3 (session 2): the fp32 config-3 change -- stage_l without captured mutable locals (no scratch), knot-major trial trajectories:
# the diag-cost test, the full GPU suite without -x, then the bench lines -> gpurun_out/r03q
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r03q; mkdir -p $O
timeout -k 10 200 python tools/debug/c3_fp32_compare.py > $O/c3.json 2> $O/c3.err; echo "c3 rc=$?" > $O/rc.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
prc=$?; echo "pytest rc=$prc" >> $O/rc.txt
[ $prc -le 1 ] || exit 0
B=/root/repo/bench.py
run() {   # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc
}
C3="--solver ilqr --limits torque-al --no-cpu-baseline"
run bench_c3 300 python $B --steps 3 --warmup 1 $C3 && \
run bench_head 300 python $B --steps 10 --warmup 3 --no-cpu-baseline && \
run bench_c4 300 python $B --steps 3 --warmup 1 --limits torque-joint-al --no-cpu-baseline && \
run bench_ilqr 200 python $B --steps 10 --warmup 3 --solver ilqr --no-cpu-baseline && \
cd /tmp && export TMPDIR=/tmp && \
run trace_c3 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 $B --steps 1 --warmup 1 $C3 && \
run trace_head 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_head -o run -- python3 $B --steps 3 --warmup 1 --no-cpu-baseline
echo "all rc=$?" >> $O/rc.txt
exit 0
