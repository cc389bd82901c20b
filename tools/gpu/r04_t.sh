# round 4 (t): hard band row-start-relative (ELL): waves walk only their longest row; hard tests, probe, bench, trace
# without the 2-link UrdfCost branch in the other instances (no scratch): hard / soft / EE / config tests,
# probe, hard bench, kernel trace, config 4 and headline bench lines
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04t; mkdir -p $O
B=/root/repo/bench.py
C4="--limits torque-joint-al --no-cpu-baseline"
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc; }
run tests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hard.py && \
run probe 300 python tools/debug/r04_hardpcg_probe.py 352 1024 && \
run hard 300 python $B --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline && \
(cd /tmp && export TMPDIR=/tmp && run kt_hard 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $B --steps 1 --warmup 0 --batch 1024 --limits torque-velocity-as --no-cpu-baseline)
exit 0
