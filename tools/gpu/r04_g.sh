# round 4 (g): hard-limit PCG residency sweep (problems per CU via the LDS allotment) + FETCH_SIZE of hard_pcg
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04g; mkdir -p $O
B=/root/repo/bench.py
for kb in 0 40 54 80 160; do
  TMPC_HARD_PCG_LDS_KB=$kb timeout -k 10 300 python $B --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline > $O/hard_lds$kb.json 2> $O/hard_lds$kb.err; echo "lds$kb rc=$?" >> $O/rc.txt
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_hard -o run -- python3 $B --steps 1 --warmup 0 --batch 1024 --limits torque-velocity-as --no-cpu-baseline > $O/fetch_hard.out 2>&1); echo "fetch rc=$?" >> $O/rc.txt
exit 0
