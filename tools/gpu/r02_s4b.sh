# full GPU suite + headline bench + rocprofv3 kernel trace (per-launch durations) for the current libtmpc.so
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/s4b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_headline.json 2> $O/bench_headline.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_trace.json 2> $O/trace.err
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
