set -o pipefail
cd /root/repo
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 120 python tools/pcg_microbench.py > $O/micro_new.jsonl 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err
