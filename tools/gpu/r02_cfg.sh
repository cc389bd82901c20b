# BASELINE configs 3 and 5 in their precision modes + config 5 on SQP (N = 128, GM QP) -> gpurun_out/r02c
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r02c; mkdir -p $O
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline > $O/c3_fp32.json 2> $O/c3_fp32.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline > $O/c3_fp64.json 2> $O/c3_fp64.err && \
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --N 128 --batch 8192 --mpc-steps 4 --pcg-warm-start --precision mixed --no-cpu-baseline > $O/c5_sqp_mixed.json 2> $O/c5_sqp_mixed.err && \
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --N 128 --batch 8192 --mpc-steps 4 --pcg-warm-start --no-cpu-baseline > $O/c5_sqp_fp64.json 2> $O/c5_sqp_fp64.err && \
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --N 128 --batch 8192 --no-cpu-baseline > $O/sqp_n128.json 2> $O/sqp_n128.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --N 128 --solver ilqr --batch 8192 --mpc-steps 4 --precision mixed --no-cpu-baseline > $O/c5_ilqr_mixed.json 2> $O/c5_ilqr_mixed.err
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
