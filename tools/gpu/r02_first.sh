set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r02a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a/gputests.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r02a/prof -o run -- python3 /root/repo/bench.py --steps 5 --warmup 2 --no-cpu-baseline > /root/repo/gpurun_out/r02a/bench_prof.json 2>/root/repo/gpurun_out/r02a/prof.err
