"""Config 3 (arm6 N = 64 iLQR + AL torque) at fp32 against the fp64 oracle fixture and the GPU's fp64 run:
per problem exit code, iterations, outer passes, max |x - x64| / max|x64|.
usage: python tools/debug/r06_fp32_probe.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_gpu_precision import _problems, _solver  # noqa: E402

d = np.load(os.path.join(ROOT, "tests", "golden", "oracle_config3_arm6_N64_ilqr_al.npz"))
N = int(d["N"])
lb, ub = float(d["lb"]), float(d["ub"])
s = _solver(6, N, {"torque": ([lb] * 6, [ub] * 6, "AUGMENTED_LAGRANGIAN")})
x, u = _problems("arm6fix", N, d["seeds"])
out = {}
for prec in ("fp64", "fp32", "mixed"):
    opts = {"max_iter_softConstraints": int(d["max_iter_softConstraints"]),
            "max_iter_SQP_DDP": int(d["max_iter_SQP_DDP"]), "precision": prec}
    r = s.iLQR_batch(x, u, N, 0.1, opts)
    rows = []
    for i in range(len(x)):
        sc = max(1.0, float(np.max(np.abs(d["x"][i]))))
        rows.append(dict(exit=int(r["exit_code"][i]), it=int(r["iter"][i]), outer=int(r["outer_iter"][i]),
                         xerr=float(np.max(np.abs(r["x"][i] - d["x"][i]))) / sc))
    out[prec] = rows
ref = [dict(exit=int(d["exit_code"][i]), it=int(d["iter"][i]), outer=int(d["outer_iter"][i])) for i in range(len(x))]
print(json.dumps(dict(oracle=ref, **out)))
for prec in ("fp64", "fp32", "mixed"):
    m = sum(out[prec][i]["exit"] == ref[i]["exit"] for i in range(len(x)))
    print(prec, "exit codes equal to the oracle's:", m, "/ 8; max xerr", max(r["xerr"] for r in out[prec]),
          "; per problem", [f"{r['exit']}/{r['it']}/{r['xerr']:.1e}" for r in out[prec]], flush=True)
