# round 4: sanity check of the tree as committed (after the reverted experiments): hard / SQP / dynamics tests,
# smoke, default bench
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04check; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hard.py tests/test_gpu_sqp.py tests/test_gpu_dynamics.py tests/test_gpu_pcg.py > $O/tests.log 2>&1; echo "tests rc=$?" > $O/rc.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?" >> $O/rc.txt
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err; echo "bench rc=$?" >> $O/rc.txt
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --batch 1024 --limits torque-velocity-as --no-cpu-baseline > $O/hard.json 2> $O/hard.err; echo "hard rc=$?" >> $O/rc.txt
exit 0
