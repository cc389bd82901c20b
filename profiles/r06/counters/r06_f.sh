#!/bin/bash
# r06 (f): PMC FETCH_SIZE / WRITE_SIZE passes of every streamed bench line (the lines' `traffic`), SQ counter
# passes of the headline k_qp and config 3's k_ilqr_backward, and the kernel-trace stats of the default bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r06f; mkdir -p $O
B=/root/repo/bench.py
C="--no-secondary --no-cpu-baseline --lockstep-steps 0 --warmup 0"
run() {   # name, timeout, command...
  local name=$1 t=$2; shift 2
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 $t "$@" > $O/$name.out 2>&1)
  local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc
}
pmc() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  run f_$name $t rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$name -o run -- python3 $B $C "$@" && \
  run w_$name $t rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$name -o run -- python3 $B $C "$@"
}
pmc head 240 --steps 20 && \
pmc c4 240 --steps 4 --limits torque-joint-al --substreams 2 && \
pmc hard 240 --steps 4 --limits torque-velocity-as --substreams 2 && \
pmc c3 300 --steps 2 --solver ilqr --limits torque-al --substreams 2 && \
pmc c3f32 300 --steps 2 --solver ilqr --limits torque-al --precision fp32 --substreams 2 && \
pmc c2 240 --steps 4 --links 3 --N 32 --batch 1024 && \
run sq1_head 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sq1_head -o run -- python3 $B $C --steps 4 && \
run sq2_head 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sq2_head -o run -- python3 $B $C --steps 4 && \
run sq1_c3 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sq1_c3 -o run -- python3 $B $C --steps 1 --solver ilqr --limits torque-al && \
run sq2_c3 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sq2_c3 -o run -- python3 $B $C --steps 1 --solver ilqr --limits torque-al && \
run sq3_c3 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sq3_c3 -o run -- python3 $B $C --steps 1 --solver ilqr --limits torque-al
echo "counters rc=$?" >> $O/rc.txt
run trace_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 $B $C --steps 2 --solver ilqr --limits torque-al --substreams 2
echo "trace_c3 rc=$?" >> $O/rc.txt
run trace 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $B --steps 20 --warmup 5
echo "all rc=$?" >> $O/rc.txt
# summaries on the box, then drop the raw per-dispatch files (the merge back is capped at 64 MiB)
S=$O/sum; mkdir -p $S
for n in head c4 hard c3 c3f32 c2; do
  [ -f $O/f_$n/run_counter_collection.csv ] && [ -f $O/w_$n/run_counter_collection.csv ] && \
    python3 tools/pmc_summary.py $O/f_$n $O/w_$n $S/pmc_$n.json "r06f $n" >> $S/log.txt 2>&1
done
[ -f $O/sq1_head/run_counter_collection.csv ] && python3 tools/sq_summary.py $S/kqp_counters.json "void tmpc::k_qp<6, 1, 768" $O/sq1_head $O/sq2_head >> $S/log.txt 2>&1
[ -f $O/sq1_c3/run_counter_collection.csv ] && python3 tools/sq_summary.py $S/ilqr_backward_counters.json "void tmpc::k_ilqr_backward<" $O/sq1_c3 $O/sq2_c3 $O/sq3_c3 >> $S/log.txt 2>&1
[ -f $O/sq1_c3/run_counter_collection.csv ] && python3 tools/sq_summary.py $S/ilqr_forward_counters.json "void tmpc::k_ilqr_forward<" $O/sq1_c3 $O/sq2_c3 $O/sq3_c3 >> $S/log.txt 2>&1
for d in trace trace_c3; do cp $O/$d/run_kernel_stats.csv $S/${d}_kernel_stats.csv 2>/dev/null; done
for n in head c4 hard c3 c3f32 c2 trace; do tail -c 4000 $O/f_$n.out > $S/f_$n.tail 2>/dev/null; done
tail -c 20000 $O/trace.out > $S/trace.out.tail 2>/dev/null
find $O -name "*.csv" ! -path "$S/*" -delete
cat $O/rc.txt
exit 0
