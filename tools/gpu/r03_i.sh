# round 3: hard-limit band ranges -- hard GPU tests, whole GPU suite, hard-limit bench line -> gpurun_out/r03i
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r03i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || exit 0
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --limits torque-velocity-as --batch 1024 --no-cpu-baseline > $O/bench_hard_as.json 2> $O/bench_hard_as.err
echo "bench_hard_as rc=$?" >> $O/rc.txt
exit 0
