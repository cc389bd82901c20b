# round 5 (p): k_hard_schur phase stamps (stamp build hS) in the hard bench workload
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05p; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
TMPC_LIBRARY=$L/libtmpc_hS.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 1024 \
  --limits torque-velocity-as --no-cpu-baseline --no-secondary > $O/schur_stamps.txt 2> $O/schur_stamps.err || exit 1
grep -c hs_stamps $O/schur_stamps.txt
