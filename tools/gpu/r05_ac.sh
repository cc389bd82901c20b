# round 5 (ac): config 3 forward-sweep stamps split (wait / prefetch issue / x stores / feedback / cost / aba / euler)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05ac; mkdir -p $O
TMPC_LIBRARY=/root/repo/trajoptmpcreference_amd/libtmpc_iS.so timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 \
  --solver ilqr --limits torque-al --no-cpu-baseline --no-secondary --no-hard-line > $O/stamps_c3.out 2> $O/stamps_c3.err || exit 1
grep ilqr_fwd $O/stamps_c3.out | head -2; grep ilqr_fwd $O/stamps_c3.out | tail -2
