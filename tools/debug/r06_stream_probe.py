"""Lock-step batch vs continuous batching (stream) on the BASELINE workloads: solves/s of each, and the
stream's status against the batch's (exit code / iterations per problem, x of the first copy bitwise).
usage: python tools/debug/r06_stream_probe.py [workload ...]   (head, c4, hard, c3, c3f32, c2, ilqr)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from trajoptmpcreference_amd import _native  # noqa: E402
from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf  # noqa: E402

WL = {
    "head": dict(n=6, N=64, B=4096, solver="PCG-SS", limits="none", prec=0),
    "c4": dict(n=6, N=64, B=4096, solver="PCG-SS", limits="torque-joint-al", prec=0),
    "hard": dict(n=6, N=64, B=4096, solver="PCG-SS", limits="torque-velocity-as", prec=0),
    "c3": dict(n=6, N=64, B=4096, solver="iLQR", limits="torque-al", prec=0),
    "c3f32": dict(n=6, N=64, B=4096, solver="iLQR", limits="torque-al", prec=1),
    "c2": dict(n=3, N=32, B=1024, solver="PCG-SS", limits="none", prec=0),
    "ilqr": dict(n=6, N=64, B=4096, solver="iLQR", limits="none", prec=0),
}


def run(name, copies=4, substreams=1):
    w = WL[name]
    n, N, B, dt = w["n"], w["N"], w["B"], 0.1
    nx, nu = 2 * n, n
    ctx = _native.Context(0)
    ctx.set_model(parse_urdf(planar_arm_urdf(n)))
    ctx.set_cost_quadratic(np.eye(nx), 100 * np.eye(nx), 0.1 * np.eye(nu), np.zeros(nx))
    lim = bench.LIMIT_PRESETS[w["limits"]]
    ctx.set_box_limits(lim)
    q0 = bench.initial_states(n, B, 0)
    x0 = np.zeros((B, nx, N))
    x0[:, :n, 0] = q0
    u0 = np.zeros((B, nu, N - 1))
    d_x0, d_u0, d_x, d_u = ctx.alloc(x0.nbytes), ctx.alloc(u0.nbytes), ctx.alloc(x0.nbytes), ctx.alloc(u0.nbytes)
    ctx.h2d(d_x0, x0)
    ctx.h2d(d_u0, u0)
    ctx.rollout_device(B, N, dt, d_x0, d_u0)
    ctx.set_options(precision=w["prec"])
    soft = bool(lim) and not bench.hard_limits(w["limits"])

    def batch(want=False):
        ctx.d2d(d_x, d_x0, x0.nbytes)
        ctx.d2d(d_u, d_u0, u0.nbytes)
        if soft:
            ctx.set_soft_state(B, N)
        if w["solver"] == "iLQR":
            return ctx.ilqr_solve_batch_device(B, N, dt, d_x, d_u, want_status=want)
        return ctx.sqp_solve_batch_device(B, N, dt, d_x, d_u, w["solver"], want_status=want)

    batch()
    ctx.synchronize()
    t = time.perf_counter()
    ex_b, it_b = batch(True)
    t_batch = time.perf_counter() - t
    xb = np.empty_like(x0)
    ctx.d2h(xb, d_x)
    P = B * copies
    d_xo, d_uo, d_st = ctx.alloc(x0.nbytes * copies), ctx.alloc(u0.nbytes * copies), ctx.alloc(P * 16)
    ctx.solve_stream_device(w["solver"], B, B, N, dt, d_x0, d_u0, B, d_xo, d_uo, d_st)   # warm-up
    ctx.synchronize()
    ctx.set_options(profile=1)
    ctx.reset_stats()
    t = time.perf_counter()
    ctx.solve_stream_device(w["solver"], P, B, N, dt, d_x0, d_u0, B, d_xo, d_uo, d_st, substreams=substreams)
    ctx.synchronize()
    t_stream = time.perf_counter() - t
    ctx.set_options(profile=0)
    kern = {}
    for k in ["qp", "hard_pcg", "hard_schur", "ilqr_backward", "ilqr_forward", "ls_terms", "ls_decide",
              "ilqr_decide", "stream_refill", "qp_grad", "ginv"]:
        c, ms = ctx.kernel_stats(k)
        if c:
            kern[k] = dict(launches=c, total_ms=round(ms, 2), avg_ms=round(ms / c, 4))
    st = np.empty((P, 4), dtype=np.int32)
    ctx.d2h(st, d_st)
    xo = np.empty((B, nx, N))
    ctx.d2d(d_x, d_xo, x0.nbytes)
    ctx.d2h(xo, d_x)
    mism = int(np.sum((st[:, 0] != np.tile(ex_b, copies)) | (st[:, 1] != np.tile(it_b, copies))))
    out = dict(workload=name, B=B, copies=copies, substreams=substreams, batch_solves_per_s=B / t_batch,
               stream_solves_per_s=P / t_stream, speedup=(P / t_stream) / (B / t_batch),
               status_mismatches=mism, x_copy0_bitwise=bool(np.array_equal(xo, xb)), kernels=kern,
               iters_mean=float(np.mean(it_b)), iters_max=int(np.max(it_b)))
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    # args: workload[:copies[:substreams]] ...
    for spec in sys.argv[1:] or ["head"]:
        parts = spec.split(":")
        run(parts[0], int(parts[1]) if len(parts) > 1 else 4, int(parts[2]) if len(parts) > 2 else 1)
