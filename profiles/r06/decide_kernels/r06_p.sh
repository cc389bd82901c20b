#!/bin/bash
# r06 (p): batched copies in the decision / hand-over kernels: full GPU suite, smoke, default bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r06p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 700 python bench.py > $O/bench_default.json 2> $O/bench_default.err
echo "rc=$?" > $O/rc.txt
