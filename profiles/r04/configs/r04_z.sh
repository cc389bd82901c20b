# round 4 (z): runtime-model check (as r04_y) + kernel traces of configs 3 and 4 (lock-step tails)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04z; mkdir -p $O
B=/root/repo/bench.py
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc; }
run tests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dynamics.py tests/test_gpu_boundary.py tests/test_gpu_ilqr.py && \
TMPC_GENERIC_MODEL=1 run generic_head 300 python $B --steps 3 --warmup 1 --no-cpu-baseline && \
TMPC_GENERIC_MODEL=1 run generic_ilqr 300 python $B --steps 3 --warmup 1 --solver ilqr --no-cpu-baseline && \
(cd /tmp && export TMPDIR=/tmp && run kt_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -o run -- python3 $B --steps 1 --warmup 0 --limits torque-joint-al --no-cpu-baseline) && \
(cd /tmp && export TMPDIR=/tmp && run kt_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o run -- python3 $B --steps 1 --warmup 0 --solver ilqr --limits torque-al --no-cpu-baseline)
exit 0
