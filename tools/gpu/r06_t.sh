#!/bin/bash
# r06 (t): the final library's headline line under rocprofv3 --kernel-trace --stats (launch durations by grid
# size next to the line's HIP-event averages), as r06_m.sh
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r06t; mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_head -o run -- python3 /root/repo/bench.py --no-secondary --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_head_under_rocprof.json 2> $O/bench_head_under_rocprof.err) && \
python3 tools/trace_summary.py $O/trace_head/run_kernel_trace.csv $O/trace_head_summary.json "tmpc::k_qp<6, 1, 768" "k_ls_terms" "k_qp_grad" > $O/trace_head_summary.txt 2>&1 && \
cp $O/trace_head/run_kernel_stats.csv $O/trace_head_kernel_stats.csv && rm -f $O/trace_head/*.csv
echo "rc=$?" > $O/rc.txt
