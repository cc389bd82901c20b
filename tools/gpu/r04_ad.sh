# round 4 (ad): k_qp_grad at three waves per SIMD (amdgpu_waves_per_eu(3): 168 VGPRs + 244 B/lane spill,
# was 232 VGPRs at two): headline / iLQR / config 4 bench, SQP tests
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04ad; mkdir -p $O
B=/root/repo/bench.py
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc; }
run head 300 python $B --steps 10 --warmup 2 --no-cpu-baseline && \
run ilqr 300 python $B --steps 5 --warmup 1 --solver ilqr --no-cpu-baseline && \
run c4 300 python $B --steps 2 --warmup 1 --limits torque-joint-al --no-cpu-baseline && \
run tests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sqp.py tests/test_gpu_dynamics.py
exit 0
