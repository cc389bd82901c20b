# round 5 (ak): rocprofv3 kernel stats of the default bench and of config 3 on the shipped library
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/r05ak; mkdir -p $O
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/def -o def -- python3 /root/repo/bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o c3 -- python3 /root/repo/bench.py --steps 2 --warmup 1 \
  --solver ilqr --limits torque-al --no-cpu-baseline --no-secondary --no-hard-line > $O/c3.json 2> $O/c3.err || exit 1
rm -f $O/def/def_kernel_trace.csv $O/c3/c3_kernel_trace.csv
head -n 8 $O/def/def_kernel_stats.csv | cut -c1-150
head -n 6 $O/c3/c3_kernel_stats.csv | cut -c1-150
