# round 4 (aa): two experiments in one binary -- k_ls_terms at 2 waves per SIMD (amdgpu_waves_per_eu(2):
# 348 B/lane of spill instead of 76 AGPRs at 1 wave), and the hard PCG without its top-of-iteration barrier
# (p formed where it is read): headline and config 4 bench, hard tests / probe / bench, SQP / soft tests
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04aa; mkdir -p $O
B=/root/repo/bench.py
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc; }
run hardtests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hard.py && \
run probe 300 python tools/debug/r04_hardpcg_probe.py 352 1024 && \
run hard 300 python $B --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline && \
run head 300 python $B --steps 10 --warmup 2 --no-cpu-baseline && \
run c4 300 python $B --steps 2 --warmup 1 --limits torque-joint-al --no-cpu-baseline && \
run tests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sqp.py tests/test_gpu_soft.py
exit 0
