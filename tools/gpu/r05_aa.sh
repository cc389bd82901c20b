# round 5 (aa): shipped build with the [2][NXU][dmax] Y layout: hard / pendulum / banded-SQP parity, default bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05aa; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py tests/test_gpu_long_horizon.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok; tail -1 $O/tests.out
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
python - <<PY
import json
d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('headline', d['value'], d.get('parity'))
h=d.get('hard_limits', {}); print('hard', h.get('value'), h.get('parity'), {k: v.get('avg_ms') for k, v in h.get('kernels', {}).items() if k in ('hard_pcg','hard_schur')})
s=d.get('secondary', {}); print('secondary', s.get('value'), s.get('parity'))
PY
