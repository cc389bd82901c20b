# config 3 (arm6 N=64 iLQR + AL torque, B=4096) kernel trace -> gpurun_out/s4d
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/s4d; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 /root/repo/bench.py --steps 1 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline > $O/bench_c3.json 2> $O/c3.err
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
