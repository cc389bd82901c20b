# final binary of the session: full GPU suite + configs 3 / 4 + headline with CPU baseline and parity
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/s4k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline > $O/bench_c3_fp64.json 2> $O/c3d.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --limits torque-joint-al --no-cpu-baseline > $O/bench_c4.json 2> $O/c4.err && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_headline.json 2> $O/bench_headline.err
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
