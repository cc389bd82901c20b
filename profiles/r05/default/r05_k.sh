# round 5 (k): the full GPU suite, smoke, and the default bench (headline + config-4 secondary + hard-limit
# line) on the shipped library
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05k; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.out 2>&1
echo "tests rc=$?"
tail -3 $O/tests.out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.out 2>&1 || { echo smoke failed; tail $O/smoke.out; exit 1; }
echo smoke ok
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo "bench rc=$?"
