# round 4: the full GPU suite on the tree as committed at the end of the round
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04suite; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "pytest rc=$?" > $O/rc.txt
exit 0
