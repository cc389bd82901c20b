# round 5 (l): the BASELINE configuration lines on the r05 library (config 2, iLQR, config 3 fp64 / fp32,
# config 5 iLQR / SQP GM mixed warm), and the default bench once more (the hard line's replay-classified
# parity)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05l; mkdir -p $O
B=/root/repo/bench.py
run() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u $B "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc" | tee -a $O/rc.txt; return $rc
}
run bench_c2 200 --steps 5 --warmup 2 --links 3 --N 32 --batch 1024 --no-cpu-baseline && \
run bench_ilqr 200 --steps 5 --warmup 2 --solver ilqr --no-cpu-baseline && \
run bench_c3 300 --steps 2 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline && \
run bench_c3_fp32 300 --steps 2 --warmup 1 --solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline && \
run bench_c5_ilqr 300 --steps 2 --warmup 1 --N 128 --batch 8192 --mpc-steps 4 --solver ilqr --no-cpu-baseline && \
run bench_c5_sqp 300 --steps 2 --warmup 1 --N 128 --batch 8192 --mpc-steps 4 --pcg-warm-start --precision mixed --no-cpu-baseline && \
run bench_default 600
exit 0
