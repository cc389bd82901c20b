# round 4 (a): SQ counters of the headline k_qp (LDS bank conflicts, LDS issue stalls, wait/busy cycles) on the
# committed binary, plus the counter list of this box -> gpurun_out/r04a
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04a; mkdir -p $O
B=/root/repo/bench.py
run() {   # name, timeout, command...
  local name=$1 t=$2; shift 2
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 $t "$@" > $O/$name.out 2>&1)
  local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc
}
(cd /tmp && timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1); echo "list rc=$?" > $O/rc.txt
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_head.json 2> $O/bench_head.err; echo "bench rc=$?" >> $O/rc.txt
run sq1 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sq1 -o run -- python3 $B --steps 1 --warmup 0 --no-cpu-baseline && \
run sq2 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o run -- python3 $B --steps 1 --warmup 0 --no-cpu-baseline
echo "all rc=$?" >> $O/rc.txt
exit 0
