# round 4 (m): kernel trace of the hard bench line (per-dispatch k_hard_pcg / k_hard_schur durations)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04m; mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 /root/repo/bench.py --steps 1 --warmup 0 --batch 1024 --limits torque-velocity-as --no-cpu-baseline > $O/kt.out 2>&1); echo "kt rc=$?" >> $O/rc.txt
exit 0
