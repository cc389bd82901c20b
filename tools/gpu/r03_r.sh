# round 3 profiling set -> gpurun_out/r03r: rocprofv3 kernel traces (per-dispatch durations) of
# configs 3 and 4 and the headline, then separate FETCH_SIZE / WRITE_SIZE PMC passes per workload
# (headline, config 3 iLQR + AL, config 4, config 5 SQP mixed / GM QP, config 5 iLQR)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/r03r; mkdir -p $O
B=/root/repo/bench.py
run() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc
}
C4="--limits torque-joint-al --no-cpu-baseline"
C3="--solver ilqr --limits torque-al --no-cpu-baseline"
C5S="--N 128 --batch 8192 --mpc-steps 4 --pcg-warm-start --precision mixed --no-cpu-baseline"
C5I="--N 128 --solver ilqr --batch 8192 --mpc-steps 4 --no-cpu-baseline"
run trace_c4 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o run -- python3 $B --steps 1 --warmup 1 $C4 && \
run trace_c3 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 $B --steps 1 --warmup 1 $C3 && \
run trace_head 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_head -o run -- python3 $B --steps 3 --warmup 1 --no-cpu-baseline && \
run trace_c5s 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5s -o run -- python3 $B --steps 1 --warmup 1 $C5S && \
run trace_c5i 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5i -o run -- python3 $B --steps 1 --warmup 1 $C5I && \
run fetch_head 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_head -o run -- python3 $B --steps 1 --warmup 0 --no-cpu-baseline && \
run write_head 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_head -o run -- python3 $B --steps 1 --warmup 0 --no-cpu-baseline && \
run fetch_c4 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c4 -o run -- python3 $B --steps 1 --warmup 0 $C4 && \
run write_c4 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c4 -o run -- python3 $B --steps 1 --warmup 0 $C4 && \
run fetch_c3 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c3 -o run -- python3 $B --steps 1 --warmup 0 $C3 && \
run write_c3 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c3 -o run -- python3 $B --steps 1 --warmup 0 $C3 && \
run fetch_c5s 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c5s -o run -- python3 $B --steps 1 --warmup 0 $C5S && \
run write_c5s 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c5s -o run -- python3 $B --steps 1 --warmup 0 $C5S && \
run fetch_c5i 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c5i -o run -- python3 $B --steps 1 --warmup 0 $C5I && \
run write_c5i 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c5i -o run -- python3 $B --steps 1 --warmup 0 $C5I
echo "all rc=$?" >> $O/rc.txt
# keep the summaries, drop the bulky per-dispatch counter files' duplicates
exit 0
