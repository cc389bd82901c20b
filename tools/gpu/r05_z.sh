# round 5 (z): k_hard_schur Y scratch layout [2][NXU][dmax] (coalesced phase-1 writes) now that phase 2
# reads full Y rows only for -[A B] x -[A B] entries: stamps, hard bench vs the shipped row-major layout
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05z; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
TMPC_LIBRARY=$L/libtmpc_hTS.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_hTS.txt 2> $O/probe_hTS.err || exit 1
grep -h "hs_stamps" $O/probe_hTS.txt | head -4
for v in hT new; do
  lib=$L/libtmpc_$v.so; [ $v = new ] && lib=$L/libtmpc.so
  for b in 1024 4096; do
    TMPC_LIBRARY=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --batch $b --limits torque-velocity-as --no-cpu-baseline \
      --no-secondary > $O/hard_${v}_B$b.json 2> $O/hard_${v}_B$b.err || exit 1
    python -c "import json;d=json.loads(open('$O/hard_${v}_B$b.json').read().strip().splitlines()[-1]);print('hard $v B$b', d['value'], d['kernels']['hard_pcg']['avg_ms'], d['kernels']['hard_schur']['avg_ms'])" | tee -a $O/probe.txt
  done
done
