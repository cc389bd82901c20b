# per-phase PCG cycle stamps of a -DTMPC_PCG_STAMPS dev library -> gpurun_out/s4exp/stamps_<lib>.txt
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/s4exp
for L in "$@"; do
  timeout -k 10 120 python tools/pcg_microbench.py --lib $L --pre SS,BJ --stamps > gpurun_out/s4exp/stamps_$(basename $L .so).txt 2>&1 || exit $?
done
