"""Dev probe: launch time of k_hard_pcg against its iteration count on real hard-limit Schur complements
(the first QP of the bench's torque-velocity-as workload, exported by tmpc_qp_hard_info), so the setup
cost and the per-iteration latency of one workgroup separate.  tol = 0 runs exactly max_iter iterations."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from trajoptmpcreference_amd import _native  # noqa: E402
from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf  # noqa: E402


def main():
    n, N, dt = 6, 64, 0.1
    nx = 2 * n
    out = {}
    model = parse_urdf(planar_arm_urdf(n))
    ctx = _native.Context(0)
    ctx.set_model(model)
    ctx.set_cost_quadratic(np.eye(nx), 100 * np.eye(nx), 0.1 * np.eye(n), np.zeros(nx))
    ctx.set_box_limits(bench.LIMIT_PRESETS["torque-velocity-as"])
    for B in (int(v) for v in sys.argv[1:] or ["352", "1024"]):
        q0 = bench.initial_states(n, B, 0)
        x0 = np.zeros((B, nx, N))
        x0[:, :n, 0] = q0
        u0 = np.zeros((B, n, N - 1))
        d_x, d_u = ctx.alloc(x0.nbytes), ctx.alloc(u0.nbytes)
        ctx.h2d(d_x, x0)
        ctx.h2d(d_u, u0)
        ctx.rollout_device(B, N, dt, d_x, d_u)
        ctx.d2h(x0, d_x)
        ctx.synchronize()
        ctx.qp_batch(x0, u0, N, dt, np.full(B, 1e-3), "PCG-SS", want_blocks=False)
        info = ctx.qp_hard_info(B, N)
        Sb, gam, dims = info["S_band"], info["gamma"], info["dim"]
        res = {"dmax": int(Sb.shape[1]), "W": int(info["W"]), "dim_mean": float(np.mean(dims)),
               "dim_max": int(np.max(dims))}
        ctx.set_options(profile=1)
        _, it = ctx.hard_pcg_batch(Sb, gam, dims, nx, "SS")
        res["natural_iters"] = {"mean": float(np.mean(it)), "max": int(np.max(it)),
                                "p50": float(np.percentile(it, 50)), "p90": float(np.percentile(it, 90))}
        for mi in (0, 1, 10, 30, 100):
            ctx.hard_pcg_batch(Sb, gam, dims, nx, "SS", tol=0.0, max_iter=mi)   # warm
            ctx.reset_stats()
            for _ in range(3):
                ctx.hard_pcg_batch(Sb, gam, dims, nx, "SS", tol=0.0, max_iter=mi)
            c, ms = ctx.kernel_stats("hard_pcg")
            res[f"ms_iter{mi}"] = ms / c
            res[f"GBps_iter{mi}"] = ctx.kernel_bytes("hard_pcg") / c / (ms / c / 1e3) / 1e9
        ctx.set_options(profile=0)
        res["us_per_iteration"] = 1e3 * (res["ms_iter100"] - res["ms_iter30"]) / 70
        out[f"B{B}"] = res
        ctx.free(d_x)
        ctx.free(d_u)
        print(json.dumps({f"B{B}": res}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
