# round 4 (w): the build with the regenerated model header: full GPU suite (incl. the nx = 14, D = 3000 hard
# PCG case), smoke, default bench, hard bench -> gpurun_out/r04w
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04w; mkdir -p $O
B=/root/repo/bench.py
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
prc=$?; echo "pytest rc=$prc" > $O/rc.txt
[ $prc -eq 0 ] || exit 0
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?" >> $O/rc.txt
timeout -k 10 240 python $B > $O/bench_default.json 2> $O/bench_default.err; echo "bench rc=$?" >> $O/rc.txt
timeout -k 10 240 python $B --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline > $O/bench_hard.json 2> $O/bench_hard.err; echo "hard rc=$?" >> $O/rc.txt
exit 0
