#!/bin/bash
# r06 (s): sub-stream count probe, K = 2 against K = 3, for the config 3 / config 4 / hard lines (alternating)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r06s; mkdir -p $O
C="--no-secondary --no-cpu-baseline --lockstep-steps 0 --warmup 2 --steps 16"
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 240 python bench.py $C "$@" > $O/$name.json 2> $O/$name.err
}
for rep in 1 2; do
  run c3_k2_$rep --solver ilqr --limits torque-al --substreams 2 && \
  run c3_k3_$rep --solver ilqr --limits torque-al --substreams 3 && \
  run c4_k2_$rep --limits torque-joint-al --substreams 2 && \
  run c4_k3_$rep --limits torque-joint-al --substreams 3 && \
  run hard_k2_$rep --limits torque-velocity-as --substreams 2 && \
  run hard_k3_$rep --limits torque-velocity-as --substreams 3 || break
done
echo "rc=$?" > $O/rc.txt
