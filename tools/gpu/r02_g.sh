set -o pipefail
cd /root/repo
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_hard.py tests/test_gpu_pendulum.py -v --timeout 200 --timeout-method thread > $O/gputests.log 2>&1; echo "rc=$?" >> $O/gputests.log
