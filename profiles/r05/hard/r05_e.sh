# round 5 (e): SQP past the fused QP's 1536 rows (banded path) and the hard suite; k_hard_pcg per-iteration
# decomposition (timing-only builds: no streamed band entries / no preconditioner / neither) on the
# probe at B = 256 (one problem per CU); kernel-trace stats of the default bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05e; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_long_horizon.py tests/test_gpu_hard.py > $O/tests.out 2>&1 || { echo tests failed; exit 1; }
echo tests ok
for v in base hnostream hnoprec hboth; do
  lib=$L/libtmpc_$v.so; [ $v = base ] && lib=$L/libtmpc.so
  TMPC_LIBRARY=$lib timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_$v.jsonl 2> $O/probe_$v.err || exit 1
  echo $v $(python -c "import json;d=json.loads(open('$O/probe_$v.jsonl').read().splitlines()[-1]);print(d['B256']['us_per_iteration'], d['B256']['ms_iter0'])") | tee -a $O/probe.txt
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run -- python3 /root/repo/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_default.out 2>&1) || exit 1
echo prof done
