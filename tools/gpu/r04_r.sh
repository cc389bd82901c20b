# round 4 (r): GM QP kernel with the P_kk^-1 rows in registers (S rows still streamed): GM tests, config 5
# SQP bench, FETCH / WRITE passes; config 3 fp32 FETCH / WRITE passes
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04r; mkdir -p $O
B=/root/repo/bench.py
C5S="--N 128 --batch 8192 --mpc-steps 4 --pcg-warm-start --precision mixed --no-cpu-baseline"
C3F="--solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline"
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc; }
run tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_long_horizon.py tests/test_gpu_mpc.py && \
run c5s 300 python $B --steps 2 --warmup 1 $C5S && \
(cd /tmp && export TMPDIR=/tmp && run fetch_c5s 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c5s -o run -- python3 $B --steps 1 --warmup 0 $C5S) && \
(cd /tmp && export TMPDIR=/tmp && run write_c5s 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c5s -o run -- python3 $B --steps 1 --warmup 0 $C5S) && \
(cd /tmp && export TMPDIR=/tmp && run fetch_c3f 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c3f -o run -- python3 $B --steps 1 --warmup 0 $C3F) && \
(cd /tmp && export TMPDIR=/tmp && run write_c3f 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c3f -o run -- python3 $B --steps 1 --warmup 0 $C3F)
exit 0
