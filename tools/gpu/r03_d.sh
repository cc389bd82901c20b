# round 3: the hard-limit GPU tests after the replay fix -> gpurun_out/r03d
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r03d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hard.py -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_hard.log 2>&1
echo "pytest rc=$?" > $O/rc.txt
exit 0
