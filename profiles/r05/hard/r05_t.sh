# round 5 (t): k_hard_pcg stair-phase stamps (stamp build), probe; hard parity on the EPS = 2 build
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05t; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hard.py tests/test_gpu_long_horizon.py > $O/tests.out 2>&1 || { echo tests failed; tail -30 $O/tests.out; exit 1; }
echo tests ok
TMPC_LIBRARY=$L/libtmpc_hS.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_hS.txt 2> $O/probe_hS.err || exit 1
grep hx_setup $O/probe_hS.txt | head -3
