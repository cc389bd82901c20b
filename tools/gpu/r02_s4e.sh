# iLQR INIT cost kernel: full GPU suite + iLQR / config 3 / config 5 bench lines
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/${S4OUT:-s4e}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --solver ilqr --no-cpu-baseline > $O/bench_ilqr.json 2> $O/ilqr.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline > $O/bench_c3_fp64.json 2> $O/c3d.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline > $O/bench_c3_fp32.json 2> $O/c3f.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --N 128 --solver ilqr --batch 8192 --mpc-steps 4 --no-cpu-baseline > $O/bench_c5_ilqr_fp64.json 2> $O/c5i.err
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
