# round 4 (ac): hard PCG streaming twelve band entries per batch (one batch for a 36-wide row past the 24 in registers)
# probe, hard bench; the runtime-model (non-bundled robot) path timed on the headline workload
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04ac; mkdir -p $O
B=/root/repo/bench.py
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc; }
run tests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hard.py && \
run probe 300 python tools/debug/r04_hardpcg_probe.py 352 1024 && \
run hard 300 python $B --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline
exit 0
