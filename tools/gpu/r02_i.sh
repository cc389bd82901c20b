set -o pipefail
cd /root/repo
O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_hard.py tests/test_gpu_pendulum.py > $O/t.log 2>&1; rc=$?; echo "rc=$rc" >> $O/t.log; exit $rc
