"""GPU-side data dump for developing the canonical-order restatements on the CPU (round 4):
  * iLQR results of the test workloads (tests/test_gpu_ilqr.py, test_gpu_configs.py config 3 / 5,
    test_gpu_precision.py fp32 config 3) -> gpurun_out/<out>/ilqr_*.npz
  * PCG-J SQP fixtures: the GPU's own run and, at every QP's iterate (the same solve stopped after j
    iterations), the QP's S blocks / gamma / lambda / PCG count -> gpurun_out/<out>/pcgj_*.npz
Usage (GPU box): python tools/debug/r04_dump.py OUTDIR
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import ARM_N, GOLDEN, arm_model, golden, quad_cost_arrays  # noqa: E402


def solver(n, N, spec=None):
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant,
                                         planar_arm_urdf)
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
    con = TrajoptConstraint(n, n, n, N)
    for kind, (lb, ub, mode) in (spec or {}).items():
        getattr(con, f"set_{kind}_limits")(ub, lb, mode)
    return TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(n)), con)


def problems(name, N, seeds):
    from oracle import sqp as osqp
    m = arm_model(name)
    xs, us = zip(*[osqp.initial_problem(m, N, 0.1, int(s)) for s in seeds])
    return np.array(xs), np.array(us)


def save_ilqr(out, tag, r, extra=None):
    d = {k: np.asarray(r[k]) for k in ("exit_code", "iter", "exit_soft", "outer_iter", "x", "u")}
    for k, v in r["trace"].items():
        d["tr_" + k] = v
    if "soft_state" in r:
        d["mu"] = r["soft_state"][0]
    d.update(extra or {})
    np.savez_compressed(os.path.join(out, f"ilqr_{tag}.npz"), **d)


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    # --- iLQR test workloads
    for name, N, B in (("arm3", 32, 16), ("arm6fix", 64, 6), ("arm2", 16, 8)):
        s = solver(ARM_N[name], N)
        x, u = problems(name, N, range(500, 500 + B))
        save_ilqr(out, f"{name}_N{N}", s.iLQR_batch(x, u, N, 0.1, {}))
    d = golden("oracle_config3_arm6_N64_ilqr_al.npz")
    N = int(d["N"])
    lb, ub = float(d["lb"]), float(d["ub"])
    opts = {"max_iter_softConstraints": int(d["max_iter_softConstraints"]),
            "max_iter_SQP_DDP": int(d["max_iter_SQP_DDP"])}
    x, u = problems("arm6fix", N, d["seeds"])
    for prec in ("fp64", "fp32"):
        s = solver(6, N, {"torque": ([lb] * 6, [ub] * 6, "AUGMENTED_LAGRANGIAN")})
        save_ilqr(out, f"config3_{prec}", s.iLQR_batch(x, u, N, 0.1, dict(opts, precision=prec)))
    d = golden("oracle_config5_arm6_N128_mpc_ilqr.npz")
    N, steps = int(d["N"]), int(d["steps"])
    x, u = problems("arm6fix", N, d["seeds"])
    s = solver(6, N)
    r = s.MPC_batch(x, u, N, 0.1, "iLQR", {}, mpc_steps=steps)
    np.savez_compressed(os.path.join(out, "ilqr_config5.npz"), **{k: np.asarray(v) for k, v in r.items()})

    # --- PCG-J SQP fixtures: the GPU run + every QP's S at the GPU's own iterate
    import glob
    for f in sorted(glob.glob(os.path.join(GOLDEN, "sqp_*_PCG-J.npz"))):
        b = os.path.basename(f)[4:-4]
        name, Ns, ss, method = b.split("_")
        N = int(Ns[1:])
        fx = np.load(f)
        n = ARM_N[name]
        s = solver(n, N)
        x0, u0 = fx["x0"][None], fx["u0"][None]
        r = s.SQP_batch(x0, u0, N, float(fx["dt"]), method, {})
        it, ex = int(r["sqp_iter"][0]), int(r["exit_sqp"][0])
        nq = it + (1 if ex == 3 else 0)
        opts = {}
        s.set_default_options(opts)
        rho, drho, f_ = opts["rho_init_SQP_DDP"], 1.0, float(opts["rho_factor_SQP_DDP"])
        dump = {"exit_sqp": ex, "sqp_iter": it, "trace_pcg": r["trace"]["pcg_iters"][0],
                "trace_ok": r["trace"]["succeeded_line_search"][0], "trace_alpha": r["trace"]["alpha"][0],
                "x": r["x"][0], "u": r["u"][0]}
        for j in range(nq):
            if j == 0:
                xj, uj = x0, u0
            else:
                rj = s.SQP_batch(x0, u0, N, float(fx["dt"]), method, {"max_iter_SQP_DDP": j})
                xj, uj = rj["x"], rj["u"]
            ctx = s._context(dict(opts))
            q = ctx.qp_batch(xj, uj, N, float(fx["dt"]), rho, method, want_blocks=True, xs=x0[:, :, 0])
            for k in ("dxul", "pcg_iters", "S_diag", "S_lo", "gamma", "P_diag"):
                dump[f"q{j}_{k}"] = q[k][0]
            dump[f"q{j}_rho"] = rho
            dump[f"q{j}_x"], dump[f"q{j}_u"] = xj[0], uj[0]
            if r["trace"]["succeeded_line_search"][0, j + 1]:
                drho = min(drho / f_, 1.0 / f_)
            else:
                drho = max(drho * f_, f_)
            rho = max(rho * drho, opts["rho_min_SQP_DDP"])
        np.savez_compressed(os.path.join(out, f"pcgj_{b}.npz"), **dump)
    print("dump done", flush=True)


if __name__ == "__main__":
    main()
