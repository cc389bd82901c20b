# round-2 profile set for the benched binary: bench lines (configs 2-5), rocprofv3 kernel-trace
# stats, and two separate PMC passes (FETCH_SIZE, WRITE_SIZE) -> gpurun_out/r02p
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r02p; mkdir -p $O
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_sqp_pcgss.json 2> $O/bench_sqp_pcgss.err && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --solver ilqr --limits torque-al --no-cpu-baseline > $O/bench_c3_ilqr_al.json 2> $O/c3.err && \
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --limits torque-joint-al --no-cpu-baseline > $O/bench_c4_sqp_al.json 2> $O/c4.err && \
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --N 128 --solver ilqr --batch 8192 --mpc-steps 4 --no-cpu-baseline > $O/bench_c5_mpc.json 2> $O/c5.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 /root/repo/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_stats.json 2> $O/stats.err && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 /root/repo/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_fetch.json 2> $O/fetch.err && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 /root/repo/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_write.json 2> $O/write.err
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
