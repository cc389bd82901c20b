# round 5 (v): per-launch kernel trace of the hard line at B = 4096 (the lock-step tail)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/r05v; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o hard -- python3 /root/repo/bench.py --steps 1 --warmup 1 \
  --batch 4096 --limits torque-velocity-as --no-cpu-baseline --no-secondary > $O/hard.json 2> $O/hard.err || exit 1
find $O/tr -name '*.csv' | head -20
