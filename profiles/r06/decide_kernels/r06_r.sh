#!/bin/bash
# r06 (r): as (q) with k_ilqr_soft_add back to its round-5 form; a second default bench for the spread
# (the batched copies of tmpc_copy.h, k_hard_ls / k_hard_dxu / k_soft_outer without dynamic array indices)
# kernel-trace stats of the streamed config 3 / config 4 / hard lines
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r06r; mkdir -p $O
B=/root/repo/bench.py
C="--no-secondary --no-cpu-baseline --lockstep-steps 0 --warmup 1"
tr() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 $t rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$name -o run -- python3 $B $C "$@" > $O/tr_$name.out 2>&1) && \
  cp $O/tr_$name/run_kernel_stats.csv $O/trace_${name}_kernel_stats.csv && rm -f $O/tr_$name/*.csv
}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 700 python bench.py > $O/bench_default.json 2> $O/bench_default.err && \
tr c3 300 --steps 4 --solver ilqr --limits torque-al --substreams 2 && \
tr c4 300 --steps 4 --limits torque-joint-al --substreams 2 && \
tr hard 300 --steps 4 --limits torque-velocity-as --substreams 2
rc=$?; [ $rc -eq 0 ] && timeout -k 10 700 python bench.py > $O/bench_default2.json 2> $O/bench_default2.err; echo "rc=$rc $?" > $O/rc.txt
