#!/bin/bash
# r06: concurrent sub-streams -- parity (stream == batch with K sub-streams) and rates for K = 1, 2, 4
set -o pipefail
mkdir -p gpurun_out/r06e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream.py > gpurun_out/r06e/tests.txt 2>&1 || { tail -40 gpurun_out/r06e/tests.txt; exit 1; }
tail -3 gpurun_out/r06e/tests.txt
timeout -k 10 700 python -u tools/debug/r06_stream_probe.py head:20:1 head:20:2 head:20:4 c4:16:1 c4:16:2 c4:16:4 hard:16:1 hard:16:2 hard:16:4 c3:16:1 c3:16:2 c3:16:4 c2:16:1 c2:16:2 c2:16:4 > gpurun_out/r06e/probe.jsonl 2>&1 || { tail -30 gpurun_out/r06e/probe.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06e/probe.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["workload"], d["copies"], d["substreams"], round(d["batch_solves_per_s"]), round(d["stream_solves_per_s"]), d["status_mismatches"], d["x_copy0_bitwise"])
PY
