# round 4 (ab): runtime models: general-topology instances for the line search and the gradient only, chain elsewhere
# runtime model, branched tree), the runtime-model path timed on the headline and iLQR workloads
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04ab; mkdir -p $O
B=/root/repo/bench.py
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc; }
run tests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dynamics.py tests/test_gpu_boundary.py tests/test_gpu_ilqr.py && \
TMPC_GENERIC_MODEL=1 run generic_head 300 python $B --steps 3 --warmup 1 --no-cpu-baseline && \
TMPC_GENERIC_MODEL=1 run generic_ilqr 300 python $B --steps 3 --warmup 1 --solver ilqr --no-cpu-baseline
exit 0
