# round 5 (m): the hard line's parity mismatch in detail (tools/debug/r05_hard_mismatch.py); k_hard_pcg's
# setup and iteration phase stamps (stamp build hS)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05m; mkdir -p $O
L=/root/repo/trajoptmpcreference_amd
timeout -k 10 300 python -u tools/debug/r05_hard_mismatch.py 5 > $O/mismatch.jsonl 2> $O/mismatch.err || { tail -20 $O/mismatch.err; exit 1; }
echo mismatch done
TMPC_LIBRARY=$L/libtmpc_hS.so timeout -k 10 200 python -u tools/debug/r04_hardpcg_probe.py 256 > $O/probe_hS.txt 2> $O/probe_hS.err || exit 1
echo stamps done
