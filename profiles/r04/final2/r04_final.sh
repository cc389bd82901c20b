# round 4, final: the round's last build end to end -> gpurun_out/r04final: full GPU suite, smoke, the
# default bench (parity leg + CPU baseline), BASELINE config lines, the hard-limit line, and the default
# bench under rocprofv3 --kernel-trace --stats
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04final; mkdir -p $O
B=/root/repo/bench.py
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
prc=$?; echo "pytest rc=$prc" > $O/rc.txt
[ $prc -eq 0 ] || exit 0
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?" >> $O/rc.txt
run() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python $B "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc
}
run bench_default 240 && \
run bench_hard 200 --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline && \
run bench_c3_fp32 200 --steps 3 --warmup 1 --solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline && \
run bench_c4 200 --steps 3 --warmup 1 --limits torque-joint-al --no-cpu-baseline && \
run bench_c5_sqp 200 --steps 2 --warmup 1 --N 128 --batch 8192 --mpc-steps 4 --pcg-warm-start --precision mixed --no-cpu-baseline && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_head -o run -- python3 $B --steps 5 --warmup 1 --no-cpu-baseline > $O/kt_head.out 2>&1); echo "kt_head rc=$?" >> $O/rc.txt
exit 0
