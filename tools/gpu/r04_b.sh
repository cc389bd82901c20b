# round 4 (b): new boundary-method GPU tests; dump GPU iLQR results of the test workloads and the PCG-J SQP
# fixtures' per-QP Schur blocks at the GPU's own iterates (tools/debug/r04_dump.py) -> gpurun_out/r04b
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_boundary.py -v --timeout 120 --timeout-method thread > $O/boundary.log 2>&1; echo "boundary rc=$?" > $O/rc.txt
timeout -k 10 400 python -u tools/debug/r04_dump.py $O > $O/dump.log 2>&1; echo "dump rc=$?" >> $O/rc.txt
exit 0
