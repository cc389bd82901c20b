# round 4 (j): hard PCG slot loops one slot at a time, z and S p in LDS; kernel-counted algorithmic bytes (hard roofline)
# hard tests (bitwise canonical parity), the hard bench line, FETCH_SIZE of hard_pcg
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04j; mkdir -p $O
B=/root/repo/bench.py
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hard.py > $O/hard_tests.log 2>&1; echo "tests rc=$?" >> $O/rc.txt
timeout -k 10 300 python $B --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline > $O/hard.json 2> $O/hard.err; echo "bench rc=$?" >> $O/rc.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_hard -o run -- python3 $B --steps 1 --warmup 0 --batch 1024 --limits torque-velocity-as --no-cpu-baseline > $O/fetch_hard.out 2>&1); echo "fetch rc=$?" >> $O/rc.txt
exit 0
