# round 3 final check of the committed binary: GPU suite, smoke(), the default bench line -> gpurun_out/r03final
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r03final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
prc=$?; echo "pytest rc=$prc" > $O/rc.txt
[ $prc -eq 0 ] || exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?" >> $O/rc.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; echo "bench rc=$?" >> $O/rc.txt
exit 0
