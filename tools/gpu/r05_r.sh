# round 5 (r): k_hard_schur S phase two entries per step (paired Y loads): hard parity, schur stamps, hard
# bench B = 1024 / 4096 for the shipped build (171 VGPRs, 2 waves per SIMD) and the 3-waves build (hW3)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05r; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_pendulum.py tests/test_gpu_long_horizon.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok
TMPC_LIBRARY=$L/libtmpc_hS.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 1024 \
  --limits torque-velocity-as --no-cpu-baseline --no-secondary > $O/schur_stamps.txt 2> $O/schur_stamps.err || exit 1
grep hs_stamps $O/schur_stamps.txt | head -4
for v in new hW3; do
  lib=$L/libtmpc_$v.so; [ $v = new ] && lib=$L/libtmpc.so
  for b in 1024 4096; do
    TMPC_LIBRARY=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
      --no-secondary > $O/hard_${v}_B$b.json 2> $O/hard_${v}_B$b.err || exit 1
    python -c "import json;d=json.loads(open('$O/hard_${v}_B$b.json').read().strip().splitlines()[-1]);print('hard $v B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'], d['kernels']['hard_schur']['avg_ms'])" | tee -a $O/probe.txt
  done
done
