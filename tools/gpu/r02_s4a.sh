# session-4 re-verification after container restore: GPU tests (incl. the new non-finite trial test) + headline bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/s4a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_headline.json 2> $O/bench_headline.err
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
