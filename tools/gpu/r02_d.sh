set -o pipefail
cd /root/repo
O=gpurun_out/r02d; mkdir -p $O
L=$PWD/trajoptmpcreference_amd
timeout -k 10 200 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_pcg.py -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1; echo "rc=$?" >> $O/gputests.log
timeout -k 10 120 python tools/pcg_microbench.py --lib $L/libtmpc_stamps.so --stamps --pre SS,BJ,J > $O/micro_stamps.jsonl 2>&1 && \
timeout -k 10 120 python tools/pcg_microbench.py --lib $L/libtmpc_rpl2.so > $O/micro_rpl2.jsonl 2>&1 && \
TMPC_LIBRARY=$L/libtmpc_rpl2.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_rpl2.json 2> $O/bench_rpl2.err
