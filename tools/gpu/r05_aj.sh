# round 5 (aj): as (ah), with the rollout feedback law reading its LDS operands ahead of the products
# suite, smoke, the default bench (headline + config-4 secondary + hard-limit line) and the BASELINE
# configuration lines
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05aj; mkdir -p $O
B=/root/repo/bench.py
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.out 2>&1
echo "tests rc=$?"
tail -n 3 $O/tests.out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.out 2>&1 || { echo smoke failed; tail $O/smoke.out; exit 1; }
echo smoke ok
run() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u $B "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc" | tee -a $O/rc.txt; return $rc
}
run bench_default 900 && \
run bench_c2 200 --steps 5 --warmup 2 --links 3 --N 32 --batch 1024 --no-cpu-baseline && \
run bench_ilqr 200 --steps 5 --warmup 2 --solver ilqr --no-cpu-baseline && \
run bench_c3 300 --steps 2 --warmup 1 --solver ilqr --limits torque-al --no-cpu-baseline && \
run bench_c3_fp32 300 --steps 2 --warmup 1 --solver ilqr --limits torque-al --precision fp32 --no-cpu-baseline && \
run bench_c5_ilqr 300 --steps 2 --warmup 1 --N 128 --batch 8192 --mpc-steps 4 --solver ilqr --no-cpu-baseline && \
run bench_c5_sqp 300 --steps 2 --warmup 1 --N 128 --batch 8192 --mpc-steps 4 --pcg-warm-start --precision mixed --no-cpu-baseline
python3 - <<PY
import json, glob
for f in sorted(glob.glob('$O/bench_*.json')):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, 'unreadable', e); continue
    extra = ''
    if 'hard_limits' in d: extra += ' hard %.1f parity %s' % (d['hard_limits'].get('value', 0), d['hard_limits'].get('parity', {}).get('mismatches'))
    if 'secondary' in d: extra += ' c4 %.1f' % d['secondary'].get('value', 0)
    print(f.split('/')[-1], round(d['value'], 1), d.get('parity', {}).get('mismatches') if isinstance(d.get('parity'), dict) else '', extra)
PY
exit 0
