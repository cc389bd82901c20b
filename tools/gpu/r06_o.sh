#!/bin/bash
# r06 (o): PMC FETCH_SIZE / WRITE_SIZE passes of the streamed config-3 fp32 line with the fp32 Riccati sweep
# on the matrix cores (k_ilqr_backward<6, float, true>), summarised on the box
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r06o; mkdir -p $O
C="--no-secondary --no-cpu-baseline --lockstep-steps 0 --warmup 0 --steps 2 --solver ilqr --limits torque-al --precision fp32 --substreams 2"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 /root/repo/bench.py $C > $O/f.out 2>&1) && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 /root/repo/bench.py $C > $O/w.out 2>&1) && \
python3 tools/pmc_summary.py $O/f $O/w $O/pmc_c3f32.json "r06o c3f32" > $O/sum.txt 2>&1
rc=$?
find $O -name "*.csv" -delete
echo "rc=$rc" > $O/rc.txt
