# round 3 (session 2): bench lines rerun with profiles/pmc shipped (.gpurunignore had dropped it), PMC
# summaries of profiles/pmc (r03/v5) in place, plus smoke() -> gpurun_out/r03t
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r03t; mkdir -p $O
B=/root/repo/bench.py
run() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python $B "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc
}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?" > $O/rc.txt
run bench_headline 400 --steps 10 --warmup 3 && \
run bench_c2_arm3 200 --steps 10 --warmup 3 --links 3 --N 32 --batch 1024 --no-cpu-baseline && \
run bench_ilqr 200 --steps 10 --warmup 3 --solver ilqr --no-cpu-baseline && \
run bench_c3_fp64 300 --steps 3 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline && \
run bench_c3_fp32 300 --steps 3 --warmup 1 --solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline && \
run bench_c4 300 --steps 3 --warmup 1 --limits torque-joint-al --no-cpu-baseline && \
run bench_c5_ilqr 300 --steps 3 --warmup 1 --N 128 --solver ilqr --batch 8192 --mpc-steps 4 --no-cpu-baseline && \
run bench_c5_sqp_mixed 300 --steps 2 --warmup 1 --N 128 --batch 8192 --mpc-steps 4 --pcg-warm-start --precision mixed --no-cpu-baseline && \
run bench_hard_as 300 --steps 2 --warmup 1 --limits torque-velocity-as --batch 1024 --no-cpu-baseline && \
run bench_converging_ee 200 --steps 10 --warmup 3 --links 2 --N 10 --cost ee --erm -100 --q0-scale 0.1 --no-cpu-baseline
echo "all rc=$?" >> $O/rc.txt
exit 0
