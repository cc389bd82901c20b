# k_qp / PCG experiment: dev libraries (arm6 only) side by side -> gpurun_out/s4exp/<tag>
#   usage: bash tools/gpu/s4_exp.sh tag lib1 [lib2 ...]
set -o pipefail
cd /root/repo
T=$1; shift
O=/root/repo/gpurun_out/s4exp/$T; mkdir -p $O
for L in "$@"; do
  n=$(basename $L .so)
  timeout -k 10 120 python tools/pcg_microbench.py --lib $L --pre SS,BJ > $O/micro_$n.json 2> $O/micro_$n.err || exit $?
  TMPC_LIBRARY=$PWD/$L timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
done
L=$1
TMPC_LIBRARY=$PWD/$L timeout -k 10 400 python -u -m pytest tests/test_gpu_pcg.py tests/test_gpu_sqp.py tests/test_gpu_configs.py -k "arm6 or config4" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
