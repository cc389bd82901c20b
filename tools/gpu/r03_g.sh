# round 3: full GPU suite + smoke + bench lines of every configuration (tools/gpu/r03_f.sh)
cd /root/repo
O=/root/repo/gpurun_out/r03g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "pytest rc=$?" > $O/rc.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?" >> $O/rc.txt
bash tools/gpu/r03_f.sh
exit 0
