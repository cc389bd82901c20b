# round 4 (k): k_hard_pcg launch time against iterations on real hard-limit S (setup vs per-iteration latency)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04k; mkdir -p $O
timeout -k 10 300 python tools/debug/r04_hardpcg_probe.py 352 1024 > $O/probe.json 2> $O/probe.err; echo "probe rc=$?" >> $O/rc.txt
exit 0
