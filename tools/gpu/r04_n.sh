# round 4 (n): hard PCG with per-row / per-wave diagonal ranges in LDS and 16 band loads in flight;
# distinct-entry byte count: hard tests, probe, hard bench, kernel trace of the hard bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hard.py > $O/hard_tests.log 2>&1; echo "tests rc=$?" >> $O/rc.txt
timeout -k 10 300 python tools/debug/r04_hardpcg_probe.py 352 1024 > $O/probe.json 2> $O/probe.err; echo "probe rc=$?" >> $O/rc.txt
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline > $O/hard.json 2> $O/hard.err; echo "bench rc=$?" >> $O/rc.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 /root/repo/bench.py --steps 1 --warmup 0 --batch 1024 --limits torque-velocity-as --no-cpu-baseline > $O/kt.out 2>&1); echo "kt rc=$?" >> $O/rc.txt
exit 0
