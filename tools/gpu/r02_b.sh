set -o pipefail
cd /root/repo
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1; echo "tests rc=$?" >> $O/gputests.log
timeout -k 10 120 python tools/pcg_microbench.py --lib gpurun_tmp_libtmpc_r01.so > $O/micro_old.jsonl 2>&1 && \
timeout -k 10 120 python tools/pcg_microbench.py > $O/micro_new.jsonl 2>&1 && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
