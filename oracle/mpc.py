"""Receding-horizon MPC loop.  TEST INFRASTRUCTURE ONLY
(see oracle/__init__.py).

The reference has no MPC loop: `runMPCExample` is called by its examples but
defined nowhere (examples/pendulum.py:28); only the hooks exist:
QuadraticCost.shift_QF_start / increase_QF (TrajoptCost.py:85-104),
BoxConstraint.shift_soft_constraint_constants (TrajoptConstraint.py:168-176,
380-387) and the MPCSolverMethods enum (TrajoptMPCReference.py:21-27).  This
module DEFINES the loop the build ships ("parity unpinned" w.r.t. the
reference); tmpc_mpc_batch is checked against it.

Per MPC step s = 0 .. steps-1, from the current trajectory (x, u):
  1. solve the horizon problem: SQP with a linear-system method, or iLQR,
     warm-started from (x, u) (the previous solution, shifted);
  2. apply the first control to the plant: x_next = integrator(x[:, 0], u[:, 0], dt);
  3. shift: x[:, k] <- x[:, k+1], u[:, k] <- u[:, k+1] (the last knot is kept),
     then x[:, 0] <- x_next;
  4. hooks: QF_start <- max(QF_start - 1, 0) when the cost has one
     (shift_QF_start(-1)); soft-limit constants shifted by one knot
     (shift_soft_constraint_constants(1), the reference's semantics).
Returns the executed states [nx][steps+1], controls [nu][steps] and the
per-step exit codes / iteration counts.
"""
import numpy as np

from . import ilqr as oilqr
from . import rbd
from . import sqp as osqp


def shift_soft(soft):
    """BoxConstraint.shift_soft_constraint_constants(1) (TrajoptConstraint.py:168-176):
    arr[:, :-1] = arr[:, 1:]; arr[:, 1:] = init."""
    if soft is None:
        return
    for lim in soft.limits:
        for arr, init in ((lim.mu, lim.o["quadratic_penalty_mu_init"]), (lim.lam, 0.0),
                          (lim.phi, lim.o["augmentated_lagrangian_phi_init"])):
            arr[:, :-1] = arr[:, 1:]
            arr[:, 1:] = init


def mpc(model, cost, x, u, N, dt, method, steps, options=None, soft=None, pcg_warm_start=False):
    """method: "iLQR" or an SQP linear-system method ("S", "PCG-SS", ...).
    pcg_warm_start: every PCG starts from the previous QP's lambda; the first QP of a step from the
    previous step's last lambda shifted by one knot (lambda_k <- lambda_{k+1}, last block kept)."""
    x = np.array(x, dtype=float)
    u = np.array(u, dtype=float)
    nx, nu = x.shape[0], u.shape[0]
    xe = np.zeros((nx, steps + 1))
    ue = np.zeros((nu, steps))
    codes = np.zeros(steps, dtype=np.int64)
    iters = np.zeros(steps, dtype=np.int64)
    xe[:, 0] = x[:, 0]
    warm = {"lam": None} if pcg_warm_start and method.startswith("PCG") else None
    for s in range(steps):
        if method == "iLQR":
            r = oilqr.ilqr(model, cost, x, u, N, dt, options, soft)
            codes[s], iters[s] = r["exit_code"], r["iter"]
        else:
            r = osqp.sqp(model, cost, x, u, N, dt, method, options, soft, warm)
            codes[s], iters[s] = r["exit_sqp"], r["sqp_iter"]
        x, u = r["x"], r["u"]
        x_next = rbd.euler(model, x[:, 0][None], u[:, 0][None], dt)[0]
        ue[:, s] = u[:, 0]
        xe[:, s + 1] = x_next
        x = np.concatenate([x[:, 1:], x[:, -1:]], axis=1)
        u = np.concatenate([u[:, 1:], u[:, -1:]], axis=1)
        x[:, 0] = x_next
        if cost.QF_start is not None:
            cost.QF_start = max(cost.QF_start - 1, 0)
        shift_soft(soft)
        if warm is not None and warm["lam"] is not None:
            L = warm["lam"].reshape(N, nx)
            warm["lam"] = np.concatenate([L[1:], L[-1:]]).reshape(-1)
    return dict(x_exec=xe, u_exec=ue, exit_codes=codes, iters=iters, x=x, u=u)
