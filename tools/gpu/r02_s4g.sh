# measurement set for the current binary -> gpurun_out/s4g: rocprofv3 kernel-trace stats (headline, iLQR),
# separate FETCH_SIZE / WRITE_SIZE PMC passes of the headline, config 2 (arm3) / 4 / 5-SQP bench lines
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/s4g; mkdir -p $O
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --links 3 --N 32 --batch 1024 --no-cpu-baseline > $O/bench_c2_arm3.json 2> $O/c2.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --limits torque-joint-al --no-cpu-baseline > $O/bench_c4.json 2> $O/c4.err && \
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --N 128 --batch 8192 --mpc-steps 4 --pcg-warm-start --precision mixed --no-cpu-baseline > $O/bench_c5_sqp_mixed.json 2> $O/c5s.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 /root/repo/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_stats.json 2> $O/stats.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_ilqr -o run -- python3 /root/repo/bench.py --steps 5 --warmup 2 --solver ilqr --no-cpu-baseline > $O/bench_stats_ilqr.json 2> $O/stats_ilqr.err && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 /root/repo/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_fetch.json 2> $O/fetch.err && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 /root/repo/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_write.json 2> $O/write.err
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
