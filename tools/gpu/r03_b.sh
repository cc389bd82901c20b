# round 3: full GPU test suite (no -x) + smoke on the ABI-6 binary -> gpurun_out/r03b
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r03b; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "pytest rc=$?" > $O/rc.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?" >> $O/rc.txt
exit 0
