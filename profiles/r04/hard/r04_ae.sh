# round 4 (ae): FETCH_SIZE / WRITE_SIZE passes of the hard-limit bench line (its roofline `traffic`)
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r04ae; mkdir -p $O
B=/root/repo/bench.py
H="--steps 1 --warmup 0 --batch 1024 --limits torque-velocity-as --no-cpu-baseline"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_hard -o run -- python3 $B $H > $O/fetch.out 2>&1); echo "fetch rc=$?" >> $O/rc.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_hard -o run -- python3 $B $H > $O/write.out 2>&1); echo "write rc=$?" >> $O/rc.txt
exit 0
