# iLQR kernel latency vs batch size (forward / backward avg per launch), fp64 and fp32
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r02ip; mkdir -p $O
for B in 64 1024 4096; do for P in fp64 fp32; do
timeout -k 10 120 python bench.py --steps 2 --warmup 1 --solver ilqr --batch $B --precision $P --no-cpu-baseline > $O/ilqr_${B}_${P}.json 2> $O/ilqr_${B}_${P}.err || exit 1
done; done
echo rc=0 > $O/rc.txt
