# round 5 (am): FETCH_SIZE / WRITE_SIZE passes of the hard-limit workload at B = 4096 on the shipped library
# (the default bench's hard_limits roofline `traffic`), separate runs
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/r05am; mkdir -p $O
B=/root/repo/bench.py
H="--steps 1 --warmup 0 --batch 4096 --limits torque-velocity-as --no-cpu-baseline --no-secondary --no-hard-line"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_hard -o run -- python3 $B $H > $O/fetch.out 2>&1 || { echo fetch failed; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_hard -o run -- python3 $B $H > $O/write.out 2>&1 || { echo write failed; exit 1; }
find $O -name 'run_counter_collection.csv' | head
