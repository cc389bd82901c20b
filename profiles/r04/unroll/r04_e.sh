# round 4 (e): iLQR replay tests on the committed binary; A/B of the full-unroll build (libtmpc_unroll.so,
# -mllvm -pragma-unroll-threshold=1000000: fp32 scratch gone, fewer VGPRs in the fp64 rollouts) -> gpurun_out/r04e
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04e; mkdir -p $O
B=/root/repo/bench.py
timeout -k 10 600 python -u -m pytest tests/test_gpu_ilqr.py tests/test_gpu_mpc.py tests/test_gpu_configs.py -v -rA --timeout 300 --timeout-method thread > $O/tests_base.log 2>&1; echo "tests_base rc=$?" > $O/rc.txt
TMPC_LIBRARY=/root/repo/trajoptmpcreference_amd/libtmpc_unroll.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dynamics.py tests/test_gpu_precision.py tests/test_gpu_ilqr.py tests/test_gpu_configs.py tests/test_gpu_pcg.py -v -rA --timeout 300 --timeout-method thread > $O/tests_unroll.log 2>&1; echo "tests_unroll rc=$?" >> $O/rc.txt
for L in libtmpc libtmpc_unroll; do
  export TMPC_LIBRARY=/root/repo/trajoptmpcreference_amd/$L.so
  timeout -k 10 200 python $B --steps 5 --warmup 1 --no-cpu-baseline > $O/head_$L.json 2> $O/head_$L.err; echo "head $L rc=$?" >> $O/rc.txt
  timeout -k 10 300 python $B --steps 3 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline > $O/c3_$L.json 2> $O/c3_$L.err; echo "c3 $L rc=$?" >> $O/rc.txt
  timeout -k 10 300 python $B --steps 3 --warmup 1 --solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline > $O/c3f32_$L.json 2> $O/c3f32_$L.err; echo "c3f32 $L rc=$?" >> $O/rc.txt
  timeout -k 10 200 python $B --steps 5 --warmup 1 --solver ilqr --no-cpu-baseline > $O/ilqr_$L.json 2> $O/ilqr_$L.err; echo "ilqr $L rc=$?" >> $O/rc.txt
  timeout -k 10 300 python $B --steps 3 --warmup 1 --limits torque-joint-al --no-cpu-baseline > $O/c4_$L.json 2> $O/c4_$L.err; echo "c4 $L rc=$?" >> $O/rc.txt
done
exit 0
