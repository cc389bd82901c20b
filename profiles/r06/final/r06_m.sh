#!/bin/bash
# r06 (m): the final default bench line, its headline under rocprofv3 --kernel-trace (launch durations by
# grid size next to the line's HIP-event averages), the full GPU suite and smoke
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r06m; mkdir -p $O
timeout -k 10 700 python bench.py > $O/bench_default.json 2> $O/bench_default.err && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_head -o run -- python3 /root/repo/bench.py --no-secondary --no-cpu-baseline --steps 20 --warmup 3 > $O/bench_head_under_rocprof.json 2> $O/bench_head_under_rocprof.err) && \
python3 tools/trace_summary.py $O/trace_head/run_kernel_trace.csv $O/trace_head_summary.json "tmpc::k_qp<6, 1, 768" "k_ls_terms" "k_qp_grad" > $O/trace_head_summary.txt 2>&1 && \
cp $O/trace_head/run_kernel_stats.csv $O/trace_head_kernel_stats.csv && rm -f $O/trace_head/*.csv && \
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
echo "rc=$?" > $O/rc.txt
