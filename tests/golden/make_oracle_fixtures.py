#!/usr/bin/env python3
"""Oracle results for the BASELINE.json configurations whose oracle runs take
minutes (arm6 N=64 with augmented-Lagrangian limits, arm6 N=128 MPC), computed
once here and stored as fixtures so that the GPU parity tests
(tests/test_gpu_configs.py) do not spend GPU-box time on the CPU restatement.

These are outputs of this repository's oracle (oracle/*.py, test
infrastructure), not of the reference -- the reference has no iLQR, no MPC loop
and cannot run vector box limits; the oracle itself is pinned
to the reference's fixtures by tests/test_oracle_golden.py.  iLQR results are
stored for both of the oracle's [K | d] solves (Cholesky and LU): where
rounding decides an integer outcome the GPU must match one of them
(tests/test_gpu_ilqr.py).

Usage:  python tests/golden/make_oracle_fixtures.py [--only config3|config4|config5|sqp128|mpc128sqp|big|hard6]
"""
import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(OUT))
sys.path.insert(0, ROOT)

# BASELINE config 3: arm6 iLQR, soft torque limits by augmented Lagrangian, N = 64
C3 = dict(N=64, B=8, seed0=800, lb=-0.5, ub=0.5, opts={"max_iter_softConstraints": 3, "max_iter_SQP_DDP": 25})
# BASELINE config 4: arm6 SQP-PCG-SS with torque and joint limits, N = 64 (reference default options)
C4 = dict(N=64, B=8, seed0=820, opts={})
# BASELINE config 5: arm6 receding-horizon MPC loop, N = 128, iLQR horizon solves
C5 = dict(N=128, B=2, seed0=900, steps=3, opts={})
# config 5 on SQP: arm6 N = 128 (1536 Schur rows, past the register-resident PCG's 1024), single
# PCG-SS solves and the MPC loop with the PCG warm start
C5S = dict(N=128, B=4, seed0=940, opts={})
C5M = dict(N=128, B=2, seed0=960, steps=3, opts={})
# the bench's hard-limit line (bench.py LIMIT_PRESETS "torque-velocity-as": ACTIVE_SET torque +-0.5 and
# velocity +-1 on every joint), arm6 N = 64, SQP PCG-SS at the reference's defaults, the oracle's banded-path
# PCG in the GPU's canonical summation order; seeds 0..7 are the bench workload's first problems
CH6 = dict(N=64, B=8, seed0=0, lb_u=-0.5, ub_u=0.5, lb_v=-1.0, ub_v=1.0)


def _model():
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    return parse_urdf(planar_arm_urdf(6))


def _cost():
    from oracle import sqp as osqp
    return osqp.QuadCost(np.eye(12), 100 * np.eye(12), 0.1 * np.eye(6), np.zeros(12))


def job_config3(args):
    seed, solve = args
    from oracle import ilqr as oilqr
    from oracle import sqp as osqp
    from oracle.soft import SoftConstraints, SoftLimit
    m = _model()
    N = C3["N"]
    x, u = osqp.initial_problem(m, N, 0.1, seed)
    lim = SoftLimit("torque", 6, N, [C3["lb"]] * 6, [C3["ub"]] * 6, "AUGMENTED_LAGRANGIAN")
    with np.errstate(all="ignore"):
        o = oilqr.ilqr(m, _cost(), x, u, N, 0.1, dict(C3["opts"]), SoftConstraints([lim]), solve=solve)
    return dict(seed=seed, solve=solve, exit_code=o["exit_code"], iter=o["iter"], exit_soft=o["exit_soft"],
                outer_iter=o["outer_iter"], x=o["x"], u=o["u"], J=o["trace"][-1]["J"],
                alpha=[t["alpha"] for t in o["trace"][1:]], mu=lim.mu.copy())


def job_config4(seed):
    from oracle import sqp as osqp
    from oracle.soft import SoftConstraints, SoftLimit
    m = _model()
    N = C4["N"]
    x, u = osqp.initial_problem(m, N, 0.1, seed)
    lims = [SoftLimit("torque", 6, N, [-0.5] * 6, [0.5] * 6, "AUGMENTED_LAGRANGIAN"),
            SoftLimit("joint", 6, N, [-1.0] * 6, [1.0] * 6, "AUGMENTED_LAGRANGIAN")]
    with np.errstate(all="ignore"):
        o = osqp.sqp(m, _cost(), x, u, N, 0.1, "PCG-SS", dict(C4["opts"]), SoftConstraints(lims))
    return dict(seed=seed, exit_sqp=o["exit_sqp"], sqp_iter=o["sqp_iter"], exit_soft=o["exit_soft"],
                outer_iter=o["outer_iter"], x=o["x"], u=o["u"], pcg_iters=list(o["pcg_iters"]),
                mu_torque=lims[0].mu.copy(), mu_joint=lims[1].mu.copy())


def job_config5(args):
    seed, solve = args
    from oracle import ilqr as oilqr
    from oracle import mpc as ompc
    from oracle import sqp as osqp
    m = _model()
    N = C5["N"]
    x, u = osqp.initial_problem(m, N, 0.1, seed)
    # the MPC loop with the chosen [K | d] solve for every horizon solve
    orig = oilqr.ilqr

    def ilqr_with(*a, **k):
        k.setdefault("solve", solve)
        return orig(*a, **k)
    ompc.oilqr.ilqr = ilqr_with
    try:
        with np.errstate(all="ignore"):
            o = ompc.mpc(m, _cost(), x, u, N, 0.1, "iLQR", C5["steps"], dict(C5["opts"]))
    finally:
        ompc.oilqr.ilqr = orig
    return dict(seed=seed, solve=solve, exit_codes=o["exit_codes"], iters=o["iters"], x_exec=o["x_exec"],
                u_exec=o["u_exec"])


def job_hard6(seed):
    from oracle import hard as ohard
    from oracle import sqp as osqp
    m = _model()
    N = CH6["N"]
    x, u = osqp.initial_problem(m, N, 0.1, seed)
    hc = ohard.HardConstraints([ohard.HardLimit("torque", 6, CH6["lb_u"], CH6["ub_u"], "ACTIVE_SET"),
                                ohard.HardLimit("velocity", 6, CH6["lb_v"], CH6["ub_v"], "ACTIVE_SET")])
    with np.errstate(all="ignore"):
        o = osqp.sqp(m, _cost(), x, u, N, 0.1, "PCG-SS", {}, hard=hc, order="canonical")
    tr = o["trace"][1:]
    return dict(seed=seed, exit_sqp=o["exit_sqp"], sqp_iter=o["sqp_iter"], x=o["x"], u=o["u"],
                pcg_iters=list(o["pcg_iters"]), alpha=[float(t["alpha"]) for t in tr],
                succeeded=[bool(t["succeeded_line_search"]) for t in tr],
                masks=[[int(v) for v in mk] for mk in o["active_masks"]], singular=list(o["singular"]))


def job_sqp128(seed):
    from oracle import sqp as osqp
    m = _model()
    N = C5S["N"]
    x, u = osqp.initial_problem(m, N, 0.1, seed)
    with np.errstate(all="ignore"):
        o = osqp.sqp(m, _cost(), x, u, N, 0.1, "PCG-SS", dict(C5S["opts"]))
    return dict(seed=seed, exit_sqp=o["exit_sqp"], sqp_iter=o["sqp_iter"], x=o["x"], u=o["u"],
                pcg_iters=list(o["pcg_iters"]), alpha=[t["alpha"] for t in o["trace"][1:]])


def job_mpc128sqp(seed):
    from oracle import mpc as ompc
    from oracle import sqp as osqp
    m = _model()
    N = C5M["N"]
    x, u = osqp.initial_problem(m, N, 0.1, seed)
    with np.errstate(all="ignore"):
        o = ompc.mpc(m, _cost(), x, u, N, 0.1, "PCG-SS", C5M["steps"], dict(C5M["opts"]), pcg_warm_start=True)
    return dict(seed=seed, exit_codes=o["exit_codes"], iters=o["iters"], x_exec=o["x_exec"], u_exec=o["u_exec"])


# SQP past the fused QP's 1536 Schur rows (the banded path, csrc/tmpc_api.cpp qp_banded): arm7 at N = 128
# (1792 rows) with PCG-SS, arm6 at N = 256 (3072 rows) with method S; the oracle's QP in the banded path's
# canonical order (oracle/hard.py: the dense KKT with no constraint rows, pcg_canonical)
CBIG = [(7, 128, 1000, "PCG-SS", {}), (7, 128, 1001, "PCG-SS", {}), (6, 256, 1010, "S", {}),
        # PCG-SS at the reference's defaults saturates at max_iter 100 on these S; a looser exit
        # tolerance makes every QP's count a decision the two runs must agree on
        (7, 128, 1002, "PCG-SS", {"exit_tolerance_linSys": 1e-3})]


def job_big(args):
    n, N, seed, method, opts = args
    from oracle import hard as ohard
    from oracle import sqp as osqp
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    m = parse_urdf(planar_arm_urdf(n))
    x, u = osqp.initial_problem(m, N, 0.1, seed)
    cost = osqp.QuadCost(np.eye(2 * n), 100 * np.eye(2 * n), 0.1 * np.eye(n), np.zeros(2 * n))
    with np.errstate(all="ignore"):
        o = osqp.sqp(m, cost, x, u, N, 0.1, method, dict(opts), hard=ohard.HardConstraints([]), order="canonical")
    return dict(n=n, N=N, seed=seed, method=method, opts=opts, exit_sqp=o["exit_sqp"], sqp_iter=o["sqp_iter"], x=o["x"],
                u=o["u"], pcg_iters=list(o["pcg_iters"]), alpha=[t["alpha"] for t in o["trace"][1:]])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--procs", type=int, default=8)
    a = ap.parse_args()
    pool = mp.get_context("fork").Pool(a.procs)
    if a.only in (None, "config3"):
        t = time.time()
        # one restatement: the [K | d] solve in the GPU's canonical order (oracle/ilqr.py chol_solve)
        jobs = [(C3["seed0"] + i, "canonical") for i in range(C3["B"])]
        rs = pool.map(job_config3, jobs, chunksize=1)
        rec = {"N": C3["N"], "seeds": np.arange(C3["seed0"], C3["seed0"] + C3["B"]), "lb": C3["lb"], "ub": C3["ub"],
               "max_iter_softConstraints": C3["opts"]["max_iter_softConstraints"],
               "max_iter_SQP_DDP": C3["opts"]["max_iter_SQP_DDP"]}
        for k in ("exit_code", "iter", "exit_soft", "outer_iter", "J"):
            rec[k] = np.array([r[k] for r in rs])
        for k in ("x", "u", "mu"):
            rec[k] = np.array([r[k] for r in rs])
        W = max(len(r["alpha"]) for r in rs)
        rec["alpha"] = np.array([r["alpha"] + [np.nan] * (W - len(r["alpha"])) for r in rs])
        np.savez_compressed(os.path.join(OUT, "oracle_config3_arm6_N64_ilqr_al.npz"), **rec)
        print(f"[oracle] config3: {time.time() - t:.0f} s; (exit, iter, soft, outer) "
              f"{list(zip(rec['exit_code'], rec['iter'], rec['exit_soft'], rec['outer_iter']))}", flush=True)
    if a.only in (None, "big"):
        t = time.time()
        for r in pool.map(job_big, CBIG, chunksize=1):
            tol = r["opts"].get("exit_tolerance_linSys")
            np.savez_compressed(os.path.join(OUT, f"oracle_big_arm{r['n']}_N{r['N']}_s{r['seed']}_{r['method']}.npz"),
                                seed=r["seed"], N=r["N"], exit_sqp=r["exit_sqp"], sqp_iter=r["sqp_iter"], x=r["x"],
                                exit_tolerance_linSys=np.nan if tol is None else tol,
                                u=r["u"], pcg_iters=np.array(r["pcg_iters"], dtype=np.int32),
                                alpha=np.array(r["alpha"]))
            print(f"[oracle] big arm{r['n']} N={r['N']} s{r['seed']} {r['method']}: exit {r['exit_sqp']} iters "
                  f"{r['sqp_iter']} pcg {r['pcg_iters']}", flush=True)
        print(f"[oracle] big: {time.time() - t:.0f} s", flush=True)
    if a.only in (None, "config4"):
        t = time.time()
        res = pool.map(job_config4, [C4["seed0"] + i for i in range(C4["B"])], chunksize=1)
        W = max(len(r["pcg_iters"]) for r in res)
        rec = {"N": C4["N"], "seeds": np.array([r["seed"] for r in res]),
               "pcg_iters": np.array([r["pcg_iters"] + [-1] * (W - len(r["pcg_iters"])) for r in res])}
        for k in ("exit_sqp", "sqp_iter", "exit_soft", "outer_iter"):
            rec[k] = np.array([r[k] for r in res])
        for k in ("x", "u", "mu_torque", "mu_joint"):
            rec[k] = np.array([r[k] for r in res])
        np.savez_compressed(os.path.join(OUT, "oracle_config4_arm6_N64_sqp_torque_joint_al.npz"), **rec)
        print(f"[oracle] config4: {time.time() - t:.0f} s; (exit, iter, soft, outer) "
              f"{list(zip(rec['exit_sqp'], rec['sqp_iter'], rec['exit_soft'], rec['outer_iter']))}", flush=True)
    if a.only in (None, "config5"):
        t = time.time()
        jobs = [(C5["seed0"] + i, "canonical") for i in range(C5["B"])]
        rs = pool.map(job_config5, jobs, chunksize=1)
        rec = {"N": C5["N"], "steps": C5["steps"], "seeds": np.arange(C5["seed0"], C5["seed0"] + C5["B"])}
        for k in ("exit_codes", "iters", "x_exec", "u_exec"):
            rec[k] = np.array([r[k] for r in rs])
        np.savez_compressed(os.path.join(OUT, "oracle_config5_arm6_N128_mpc_ilqr.npz"), **rec)
        print(f"[oracle] config5: {time.time() - t:.0f} s; iters {rec['iters'].tolist()}", flush=True)
    if a.only in (None, "sqp128"):
        t = time.time()
        res = pool.map(job_sqp128, [C5S["seed0"] + i for i in range(C5S["B"])], chunksize=1)
        W = max(len(r["pcg_iters"]) for r in res)
        Wa = max(len(r["alpha"]) for r in res)
        rec = {"N": C5S["N"], "seeds": np.array([r["seed"] for r in res]),
               "pcg_iters": np.array([r["pcg_iters"] + [-1] * (W - len(r["pcg_iters"])) for r in res]),
               "alpha": np.array([r["alpha"] + [np.nan] * (Wa - len(r["alpha"])) for r in res])}
        for k in ("exit_sqp", "sqp_iter", "x", "u"):
            rec[k] = np.array([r[k] for r in res])
        np.savez_compressed(os.path.join(OUT, "oracle_arm6_N128_sqp_pcgss.npz"), **rec)
        print(f"[oracle] sqp128: {time.time() - t:.0f} s; (exit, iter) "
              f"{list(zip(rec['exit_sqp'], rec['sqp_iter']))}", flush=True)
    if a.only in (None, "hard6"):
        t = time.time()
        res = pool.map(job_hard6, [CH6["seed0"] + i for i in range(CH6["B"])], chunksize=1)
        W = max(len(r["pcg_iters"]) for r in res)
        rec = {"N": CH6["N"], "seeds": np.array([r["seed"] for r in res]),
               "lb_u": CH6["lb_u"], "ub_u": CH6["ub_u"], "lb_v": CH6["lb_v"], "ub_v": CH6["ub_v"],
               "pcg_iters": np.array([r["pcg_iters"] + [-1] * (W - len(r["pcg_iters"])) for r in res]),
               "alpha": np.array([r["alpha"] + [np.nan] * (W - len(r["alpha"])) for r in res]),
               "succeeded": np.array([r["succeeded"] + [False] * (W - len(r["succeeded"])) for r in res]),
               "singular": np.array([r["singular"] + [False] * (W - len(r["singular"])) for r in res]),
               "masks": np.array([r["masks"] + [[0] * CH6["N"]] * (W - len(r["masks"])) for r in res],
                                 dtype=np.uint64)}
        for k in ("exit_sqp", "sqp_iter", "x", "u"):
            rec[k] = np.array([r[k] for r in res])
        np.savez_compressed(os.path.join(OUT, "oracle_hard_arm6_N64_torque_velocity_as.npz"), **rec)
        print(f"[oracle] hard6: {time.time() - t:.0f} s; (exit, iter) "
              f"{list(zip(rec['exit_sqp'], rec['sqp_iter']))}", flush=True)
    if a.only in (None, "mpc128sqp"):
        t = time.time()
        res = pool.map(job_mpc128sqp, [C5M["seed0"] + i for i in range(C5M["B"])], chunksize=1)
        rec = {"N": C5M["N"], "steps": C5M["steps"], "seeds": np.array([r["seed"] for r in res])}
        for k in ("exit_codes", "iters", "x_exec", "u_exec"):
            rec[k] = np.array([r[k] for r in res])
        np.savez_compressed(os.path.join(OUT, "oracle_config5_arm6_N128_mpc_sqp_pcgss.npz"), **rec)
        print(f"[oracle] mpc128sqp: {time.time() - t:.0f} s; iters {rec['iters'].tolist()}", flush=True)
    pool.close()


if __name__ == "__main__":
    main()
