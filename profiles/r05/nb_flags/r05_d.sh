# round 5 (d): neighbour-flag variants (TMPC_DEV_NJ=6 kernels builds) A/B against full barriers; PMC
# FETCH / WRITE passes of the headline on the shipped library; the default bench (headline + config-4
# secondary, CPU baseline, parity)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05d; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
for rep in 1 2; do
  for v in nb0 nb3s0 nb1s0 nb2s0 nb2s1; do
    TMPC_LIBRARY=$L/libtmpc_$v.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --no-secondary > $O/ab_${v}_$rep.json 2> $O/ab_${v}_$rep.err || exit 1
    python -c "import json;d=json.loads(open('$O/ab_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', $rep, d['value'], d['kernels']['qp']['avg_ms'])" | tee -a $O/ab.txt
  done
done
B=/root/repo/bench.py
H="--steps 3 --warmup 1 --no-cpu-baseline --no-secondary"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_head -o run -- python3 $B $H > $O/fetch.out 2>&1) || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_head -o run -- python3 $B $H > $O/write.out 2>&1) || exit 1
echo pmc done
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo "default bench rc=$?"
