#!/bin/bash
# r06: first full default bench with continuous batching and every BASELINE config line
set -o pipefail
mkdir -p gpurun_out/r06c
export TMPDIR=/tmp
timeout -k 10 580 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06c/bench.json 2> gpurun_out/r06c/bench.err || { tail -30 gpurun_out/r06c/bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06c/bench.json"))
def short(l):
    return {k: l.get(k) for k in ("value", "ms_per_step", "mode", "stream_check", "lockstep", "batch_iterations", "parity")}
print(json.dumps({"headline": short(d), "pcie": d.get("value_pcie_inclusive"), "cpu": d.get("cpu_baseline", {}) and d["cpu_baseline"]["value"]}))
for k in ("secondary", "hard_limits", "config2", "config3", "config3_fp32", "config5"):
    if k in d:
        print(k, json.dumps(short(d[k]))[:1500])
PY
