# round 3: iLQR phase stamps of the final sweeps (diagnostic library libtmpc_istamps.so, -DTMPC_ILQR_STAMPS)
# on config 3 -- the "after" of profiles/r03/v2/ilqr_stamps_before -> gpurun_out/r03x
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r03x; mkdir -p $O
TMPC_LIBRARY=/root/repo/trajoptmpcreference_amd/libtmpc_istamps.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --solver ilqr --limits torque-al --no-cpu-baseline > $O/stamps_c3.out 2> $O/stamps_c3.err
echo "stamps_c3 rc=$?" > $O/rc.txt
exit 0
