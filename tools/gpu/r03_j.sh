# round 3: hard-limit band ranges (GPU suite + hard bench line) and the iLQR phase stamps of the
# current sweeps (diagnostic library libtmpc_istamps.so) on config 3 -> gpurun_out/r03j
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r03j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || exit 0
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --limits torque-velocity-as --batch 1024 --no-cpu-baseline > $O/bench_hard_as.json 2> $O/bench_hard_as.err
echo "bench_hard_as rc=$?" >> $O/rc.txt
TMPC_LIBRARY=/root/repo/trajoptmpcreference_amd/libtmpc_istamps.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --solver ilqr --limits torque-al --no-cpu-baseline > $O/stamps_c3.out 2> $O/stamps_c3.err
echo "stamps_c3 rc=$?" >> $O/rc.txt
exit 0
