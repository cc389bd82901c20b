set -o pipefail
cd /root/repo
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_mpc.py tests/test_gpu_comm.py -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1; echo "rc=$?" >> $O/gputests.log
