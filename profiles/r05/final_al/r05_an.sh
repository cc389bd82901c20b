# round 5 (an): the default bench on the shipped library with the hard line's PMC summary in place
set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out/r05an; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
python3 -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);h=d['hard_limits'];print('default', round(d['value'],1), d['parity']['mismatches'], 'hard', round(h['value'],1), h['roofline']['traffic'], h['roofline'].get('hbm_GBps'), 'c4', round(d['secondary']['value'],1))"
