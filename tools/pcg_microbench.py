"""PCG kernel microbenchmark: tmpc_pcg_batch on B synthetic arm6 (nx = 12,
N = 64) Schur complements with a forced iteration count (tol = 0), timed
with the library's own HIP events (options.profile).  Prints one JSON line
per (library, preconditioner): us per PCG iteration per problem and per CU.

The blocks are the reference's first-QP S of the arm6 N=64 fixture
(tests/golden/qp_arm6fix_N64.npz) scaled per problem, so every problem runs
the same 100 iterations.  Usage (GPU box):
    python tools/pcg_microbench.py [--lib path.so ...] [--batch 4096]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pre", default="SS,BJ,J")
    ap.add_argument("--stamps", action="store_true", help="library built with -DTMPC_PCG_STAMPS")
    a = ap.parse_args()
    from trajoptmpcreference_amd import _native
    lib = os.path.abspath(a.lib) if a.lib else _native.LIB_PATH
    _native.load_library(lib)
    ctx = _native.Context(0)
    ctx.set_options(profile=1)
    d = np.load(os.path.join(ROOT, "tests", "golden", "qp_arm6fix_N64.npz"))
    rng = np.random.default_rng(0)
    B = a.batch
    sc = rng.uniform(0.5, 2.0, B)
    Sd = np.ascontiguousarray(d["S_diag"][None] * sc[:, None, None, None])
    Sl = np.ascontiguousarray(d["S_lo"][None] * sc[:, None, None, None])
    g = np.ascontiguousarray(d["gamma"][None] * rng.uniform(0.5, 2.0, (B, 1)))
    ncu = 256
    for pre in a.pre.split(","):
        best = None
        for _ in range(a.reps):
            ctx.reset_stats()
            lam, it, tn, _, _ = ctx.pcg_batch(Sd, Sl, g, precond=pre, tol=0.0, max_iter=a.iters, trace=a.stamps)
            n, ms = ctx.kernel_stats("pcg")
            best = ms if best is None else min(best, ms)
        iters = int(it[0])
        per_iter_us = best * 1e3 / iters
        waves = -(-B // ncu)
        print(json.dumps({"lib": os.path.basename(lib), "pre": pre, "B": B, "iters": iters, "kernel_ms": best,
                          "us_per_iter_per_cu": per_iter_us / waves,
                          "lam_checksum": float(np.sum(lam[:, :12])), "lam0": float(lam[0, 0])}), flush=True)
        if a.stamps:
            # per-phase cycles per iteration, first / last wave, problems 0 and B-1
            for b in (0, B - 1):
                for w, off in (("first", 0), ("last", 16)):
                    c = tn[b, off:off + 11] / iters
                    print(json.dumps({"pre": pre, "b": b, "wave": w, "cycles_per_iter_by_phase": [round(v) for v in c],
                                      "total": round(float(np.sum(c)))}), flush=True)


if __name__ == "__main__":
    main()
