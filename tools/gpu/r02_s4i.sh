# final headline line (CPU baseline, parity, roofline with the r02 v10 PMC traffic) + smoke -> gpurun_out/s4i
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/s4i; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_headline.json 2> $O/bench_headline.err
rc=$?; echo "rc=$rc" > $O/rc.txt; exit $rc
