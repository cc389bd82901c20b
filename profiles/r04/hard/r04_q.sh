# round 4 (q): hard PCG on 1024 threads with the LDS preconditioner-block cache + GM rows lane-major 16-byte pairs
# FETCH / WRITE passes
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04q; mkdir -p $O
B=/root/repo/bench.py
C5S="--N 128 --batch 8192 --mpc-steps 4 --pcg-warm-start --precision mixed --no-cpu-baseline"
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "$name rc=$rc" >> $O/rc.txt; return $rc; }
run tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hard.py tests/test_gpu_long_horizon.py tests/test_gpu_mpc.py && \
run probe 300 python tools/debug/r04_hardpcg_probe.py 352 1024 && \
run hard 300 python $B --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline && \
(cd /tmp && export TMPDIR=/tmp && run kt_hard 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $B --steps 1 --warmup 0 --batch 1024 --limits torque-velocity-as --no-cpu-baseline) && \
run c5s 300 python $B --steps 2 --warmup 1 $C5S && \
(cd /tmp && export TMPDIR=/tmp && run fetch_c5s 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c5s -o run -- python3 $B --steps 1 --warmup 0 $C5S) && \
(cd /tmp && export TMPDIR=/tmp && run write_c5s 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_c5s -o run -- python3 $B --steps 1 --warmup 0 $C5S)
exit 0
