# round 3, first GPU call: full GPU test suite on the ABI-6 binary (hard-limit parity rework, method N,
# singular flags), smoke, and a headline bench line -> gpurun_out/r03a
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r03a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc1=$?
echo "pytest rc=$rc1" > $O/rc.txt
if [ $rc1 -eq 0 ] || [ $rc1 -eq 1 ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_headline.json 2> $O/bench_headline.err
  rc2=$?
  echo "bench rc=$rc2" >> $O/rc.txt
fi
exit 0
