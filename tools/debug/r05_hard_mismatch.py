"""Dev probe: the bench hard line's parity mismatch (problem 5 of the first 16, torque-velocity-as):
the GPU's and the oracle's integers side by side, and at the first differing QP the GPU's own iterate
re-solved with the canonical-order PCG on its own S."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from oracle import hard as ohard  # noqa: E402
from trajoptmpcreference_amd import _native  # noqa: E402
from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf  # noqa: E402


def main():
    n, N, dt = 6, 64, 0.1
    nx = 2 * n
    probs = [int(v) for v in sys.argv[1:]] or [5]
    ctx = _native.Context(0)
    ctx.set_model(parse_urdf(planar_arm_urdf(n)))
    ctx.set_cost_quadratic(np.eye(nx), 100 * np.eye(nx), 0.1 * np.eye(n), np.zeros(nx))
    ctx.set_box_limits(bench.LIMIT_PRESETS["torque-velocity-as"])
    for p in probs:
        from oracle import sqp as osqp
        x0, u0 = osqp.initial_problem(parse_urdf(planar_arm_urdf(n)), N, dt, p)
        ref = bench._cpu_solve_hard((p, n, N))
        gr = ctx.sqp_solve_batch(x0[None], u0[None], N, dt, "PCG-SS")
        ex, it = int(gr["exit_sqp"][0]), int(gr["sqp_iter"][0])
        g = [int(v) for v in gr["trace"]["pcg_iters"][0, 1:it + 2]]
        out = {"problem": p, "gpu": [ex, it, g], "oracle": [ref["exit_sqp"], ref["sqp_iter"], ref["pcg_iters"]],
               "alpha_gpu": [float(v) for v in gr["trace"]["alpha"][0, :it + 2]],
               "succ_gpu": [int(v) for v in gr["trace"]["succeeded_line_search"][0, :it + 2]],
               "rho_gpu": [float(v) for v in gr["trace"]["rho"][0, :it + 2]]}
        out["alpha_oracle"] = ref["alpha"]
        out["succ_oracle"] = [int(v) for v in ref["succeeded"]]
        out["classified"] = bench.classify_hard_mismatch(ctx, x0[None], u0[None], N, dt, "PCG-SS", gr, 0, ref)
        j = next((q for q in range(min(len(g), len(ref["pcg_iters"]))) if g[q] != ref["pcg_iters"][q]), None)
        out["first_diff"] = j
        if False:
            # the details: the QP at the GPU's iterate j with every rho candidate
            o = ctx.options
            xi, ui = x0[None], u0[None]
            if j > 0:
                keep = o.max_iter_SQP_DDP
                ctx.set_options(max_iter_SQP_DDP=j)
                rj = ctx.sqp_solve_batch(xi, ui, N, dt, "PCG-SS", with_trace=False)
                ctx.set_options(max_iter_SQP_DDP=keep)
                xi, ui = rj["x"], rj["u"]
            det = []
            for rho in sorted(set(out["rho_gpu"])):
                q = ctx.qp_batch(xi, ui, N, dt, np.array([rho]), "PCG-SS", want_blocks=False, xs=x0[None, :, 0])
                info = ctx.qp_hard_info(1, N)
                D, W = int(info["dim"][0]), int(info["W"])
                S = np.zeros((D, D))
                for off in range(2 * W + 1):
                    a = np.arange(D)
                    c = a - W + off
                    ok = (c >= 0) & (c < D)
                    S[a[ok], c[ok]] = info["S_band"][0][a[ok], off]
                _, it_c = ohard.pcg_canonical(S, info["gamma"][0, :D], nx, "SS", o.exit_tolerance_linSys,
                                              o.max_iter_linSys)
                det.append({"rho": rho, "gpu_qp": int(q["pcg_iters"][0]), "canonical": int(it_c), "D": D})
            out["replay"] = det
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
