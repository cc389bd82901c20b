# round 5 (ab): config 3 (iLQR + AL) where the time goes now: per-knot phase stamps of the sweeps
# (libtmpc_iS.so, -DTMPC_ILQR_STAMPS) and a per-launch kernel trace of one solve
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/r05ab; mkdir -p $O
TMPC_LIBRARY=/root/repo/trajoptmpcreference_amd/libtmpc_iS.so timeout -k 10 300 python3 /root/repo/bench.py --steps 1 --warmup 0 \
  --solver ilqr --limits torque-al --no-cpu-baseline --no-secondary --no-hard-line > $O/stamps_c3.out 2> $O/stamps_c3.err || exit 1
grep -c stamps $O/stamps_c3.out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o c3 -- python3 /root/repo/bench.py --steps 1 --warmup 1 \
  --solver ilqr --limits torque-al --no-cpu-baseline --no-secondary --no-hard-line > $O/c3.json 2> $O/c3.err || exit 1
tail -c 400 $O/c3.json
