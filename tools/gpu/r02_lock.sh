# lock-step statistics of the soft-constraint configs (3: iLQR + AL torque, 4: SQP PCG-SS + AL torque/joint)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r02l; mkdir -p $O
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --limits torque-joint-al --no-cpu-baseline > $O/c4.json 2> $O/c4.err
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
