set -o pipefail
cd /root/repo
O=gpurun_out/r02h; mkdir -p $O
timeout -k 10 200 python tools/debug/pendulum_step.py > $O/step.log 2>&1; echo "rc=$?" >> $O/step.log
