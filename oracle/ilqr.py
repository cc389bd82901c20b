"""iLQR (SURVEY §8a rows a18 backward Riccati sweep / a19 forward sweep +
line search).  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference has NO iLQR: `MPCSolverMethods.iLQR` is an enum value only
(TrajoptMPCReference.py:21-27).  This module DEFINES the
algorithm this build ships, on the reference's own plugin hooks and option
keys, so it is "parity unpinned" with respect to the reference; the GPU
path (tmpc_ilqr_solve_batch) is checked against this restatement.

Hooks and options used exactly as the SQP uses them:
  * dynamics: TrajoptPlant.integrator (Euler, :83-108) and its gradient
    A_k, B_k (return_gradient=True);
  * cost: QuadraticCost value / gradient / hessian (TrajoptCost.py:24-104);
    soft limits (oracle/soft.py) add their value to J, their jacobian to
    l_xu and their per-type outer products to l_xuxu, as formKKTSystemBlocks
    does (TrajoptMPCReference.py:220-225);
  * *_SQP_DDP option keys (:99-109): rho init / factor / min / max, alpha
    factor / min, expected-reduction window, exit tolerance, max iterations;
    the rho schedule and exit codes are reduce_regularization /
    check_for_exit_or_error (:457-481); the soft-constraint outer loop is
    check_and_update_soft_constraints (:483-508).

Algorithm (per iteration):
  backward, k = N-2 .. 0, from V_x = l_x(N-1), V_xx = l_xx(N-1):
    Q_x  = l_x + A^T V_x          Q_u  = l_u + B^T V_x
    Q_xx = l_xx + A^T V_xx A      Q_uu = l_uu + B^T V_xx B + rho I
    Q_ux = l_ux + B^T V_xx A
    K = -Q_uu^-1 Q_ux,  d = -Q_uu^-1 Q_u          (Cholesky of Q_uu; failure = error)
    dV1 += d^T Q_u,  dV2 += 1/2 d^T Q_uu d
    V_x = Q_x + Q_ux^T d,  V_xx = Q_xx + Q_ux^T K,  V_xx <- (V_xx + V_xx^T) / 2
  forward, alpha = 1, f, f^2, ... while alpha > alpha_min:
    x^_0 = x_0,  u^_k = u_k + alpha d_k + K_k (x^_k - x_k),  x^_{k+1} = f(x^_k, u^_k)
    accept iff  ratio = (J - J^) / (-alpha (dV1 + alpha dV2))  in [exp_red_min, exp_red_max]
  on accept: rho <- reduce_regularization; on failure (no alpha accepted, or Q_uu not
  positive definite): the error branch of check_for_exit_or_error.
The starting trajectory is the rollout of u from x[:, 0] (iLQR iterates stay
dynamically feasible, so the constraint violation c is 0 throughout).
"""
import numpy as np

from . import rbd
from .sqp import default_options, total_cost


def rollout(model, x0, u, dt):
    N = u.shape[1] + 1
    x = np.zeros((x0.shape[0], N))
    x[:, 0] = x0
    for k in range(N - 1):
        x[:, k + 1] = rbd.euler(model, x[:, k][None], u[:, k][None], dt)[0]
    return x


def derivatives(cost, x, u, N, soft=None):
    """l_x, l_u, l_xx, l_uu per knot (l_ux = 0 for QuadraticCost; soft limits keep x / u decoupled)."""
    nx, nu = x.shape[0], u.shape[0]
    lx, lu, lxx, luu = [], [], [], []
    for k in range(N):
        uk = u[:, k] if k < N - 1 else None
        g = np.asarray(cost.gradient(x[:, k], uk, k), dtype=float).reshape(-1)
        H = np.asarray(cost.hessian(uk is None, k), dtype=float)
        if soft is not None:
            js = soft.jacobians(x[:, k], uk, k, N, nx + nu if uk is not None else nx)
            if js:
                g = g + sum(js)
                H = H + sum(np.outer(j, j) for j in js)
        lx.append(g[:nx])
        lxx.append(H[:nx, :nx])
        if uk is not None:
            lu.append(g[nx:])
            luu.append(H[nx:, nx:])
    return lx, lu, lxx, luu


def chol_solve(Quu, rhs):
    """[K | d] = Q_uu^-1 rhs in ONE canonical order -- the GPU's (k_ilqr_backward, tmpc_ilqr.hip):
    LAPACK dpotf2's Cholesky Q_uu = L L^T with the column below each pivot scaled by the pivot's
    reciprocal (numpy.linalg.cholesky's form), then per right-hand-side column the forward and back
    substitutions, each sum sequential in m and scaled by the same reciprocal.  Returns None when Q_uu
    is not positive definite (a pivot <= 0: the backward pass fails, as LinAlgError does).  The GPU
    contracts each update into a fused multiply-add; the integers (exit codes, iteration and line-search
    counts, alpha paths) of every tested workload are identical to this restatement's."""
    n = Quu.shape[0]
    L = np.zeros((n, n))
    ri = np.zeros(n)
    for j in range(n):
        s = Quu[j, j]
        for m in range(j):
            s = s - L[j, m] * L[j, m]
        if not s > 0:
            return None
        L[j, j] = np.sqrt(s)
        ri[j] = 1.0 / L[j, j]
        for i in range(j + 1, n):
            v = Quu[i, j]
            for m in range(j):
                v = v - L[i, m] * L[j, m]
            L[i, j] = v * ri[j]
    y = np.array(rhs, dtype=np.float64, copy=True)
    for i in range(n):                       # L y = rhs (all columns at once, the same order per column)
        v = y[i].copy()
        for m in range(i):
            v = v - L[i, m] * y[m]
        y[i] = v * ri[i]
    for i in range(n - 1, -1, -1):           # L^T z = y
        v = y[i].copy()
        for m in range(i + 1, n):
            v = v - L[m, i] * y[m]
        y[i] = v * ri[i]
    return y


def backward(A, B, lx, lu, lxx, luu, rho, solve="canonical"):
    """Riccati sweep; returns (K, d, dV1, dV2, ok).  [K | d] by chol_solve (the one canonical order the
    GPU follows); solve = "lu" (np.linalg.solve) and "numpy-cholesky" (np.linalg.cholesky + two
    np.linalg.solve) are kept only for the history of tests/golden/make_oracle_fixtures.py."""
    N = len(lx)
    nu = lu[0].shape[0]
    Vx = lx[N - 1].copy()
    Vxx = lxx[N - 1].copy()
    K = [None] * (N - 1)
    d = [None] * (N - 1)
    dV1 = dV2 = 0.0
    for k in range(N - 2, -1, -1):
        Ak, Bk = A[k], B[k]
        Qx = lx[k] + Ak.T @ Vx
        Qu = lu[k] + Bk.T @ Vx
        Qxx = lxx[k] + Ak.T @ (Vxx @ Ak)
        Quu = luu[k] + Bk.T @ (Vxx @ Bk) + rho * np.eye(nu)
        Qux = Bk.T @ (Vxx @ Ak)
        rhs = np.hstack([Qux, Qu[:, None]])
        if solve == "canonical":
            sol = chol_solve(Quu, rhs)
            if sol is None:
                return None, None, 0.0, 0.0, False
        else:
            try:
                L = np.linalg.cholesky(Quu)
            except np.linalg.LinAlgError:
                return None, None, 0.0, 0.0, False
            sol = np.linalg.solve(L.T, np.linalg.solve(L, rhs)) if solve == "numpy-cholesky" else \
                np.linalg.solve(Quu, rhs)
        K[k] = -sol[:, :-1]
        d[k] = -sol[:, -1]
        dV1 += d[k] @ Qu
        dV2 += 0.5 * d[k] @ (Quu @ d[k])
        Vx = Qx + Qux.T @ d[k]
        Vxx = Qxx + Qux.T @ K[k]
        Vxx = 0.5 * (Vxx + Vxx.T)
    return K, d, dV1, dV2, True


def forward(model, x, u, K, d, alpha, dt):
    N = x.shape[1]
    xn = np.zeros_like(x)
    un = np.zeros_like(u)
    xn[:, 0] = x[:, 0]
    for k in range(N - 1):
        un[:, k] = u[:, k] + alpha * d[k] + K[k] @ (xn[:, k] - x[:, k])
        xn[:, k + 1] = rbd.euler(model, xn[:, k][None], un[:, k][None], dt)[0]
    return xn, un


def step(model, cost, x, u, N, dt, rho, J, o, soft=None, solve="canonical"):
    """One iLQR iteration from the iterate (x, u) with cost J and regularisation rho: backward sweep, then
    the line search alpha = 1, f, f^2, ... until the ratio test accepts or alpha <= alpha_min.  Returns
    dict(x, u, J, error, delta_J, succeeded, ls, alpha, ratio, dV1, trials) -- the new iterate on acceptance,
    the old one otherwise (error: Q_uu not positive definite, or no alpha accepted); trials lists each
    line-search trial's (alpha, J_new, ratio)."""
    A, B = rbd.euler_gradient(model, x[:, :N - 1].T, u.T, dt)
    lx, lu, lxx, luu = derivatives(cost, x, u, N, soft)
    K, d, dV1, dV2, ok = backward(A, B, lx, lu, lxx, luu, rho, solve)
    if not ok:
        return dict(x=x, u=u, J=J, error=True, delta_J=0.0, succeeded=False, ls=0, alpha=0.0, ratio=None, dV1=None,
                    trials=[])
    alpha, ls = 1, 0
    trials = []
    while True:
        xn, un = forward(model, x, u, K, d, alpha, dt)
        J_new = total_cost(cost, xn, un, N, soft)
        delta_J = J - J_new
        with np.errstate(divide="ignore", invalid="ignore"):
            ratio = np.float64(delta_J) / np.float64(-alpha * (dV1 + alpha * dV2))
        trials.append((alpha, J_new, ratio))
        if ratio >= o["expected_reduction_min_SQP_DDP"] and ratio <= o["expected_reduction_max_SQP_DDP"]:
            return dict(x=xn, u=un, J=J_new, error=False, delta_J=delta_J, succeeded=True, ls=ls, alpha=alpha,
                        ratio=ratio, dV1=dV1, trials=trials)
        if alpha > o["alpha_min_SQP_DDP"]:
            alpha *= o["alpha_factor_SQP_DDP"]
            ls += 1
        else:
            return dict(x=x, u=u, J=J, error=True, delta_J=delta_J, succeeded=False, ls=ls, alpha=alpha,
                        ratio=ratio, dV1=dV1, trials=trials)


def ilqr(model, cost, x, u, N, dt, options=None, soft=None, solve="canonical"):
    """Returns dict(x, u, exit_code, exit_soft, outer_iter, iter, trace)."""
    o = default_options(options)
    x = rollout(model, np.array(x, dtype=float)[:, 0], np.array(u, dtype=float), dt)
    u = np.array(u, dtype=float)
    outer = 0
    exit_soft = 0
    while True:
        rho = o["rho_init_SQP_DDP"]
        drho = 1
        J = total_cost(cost, x, u, N, soft)
        trace = [dict(outer_iteration=outer, iteration=0, line_search_iteration=0, alpha=1, rho=rho, J=J,
                      dV1=None, reduction_ratio=None, succeeded_line_search=False)]
        it = 0
        exit_code = 0
        while True:
            st = step(model, cost, x, u, N, dt, rho, J, o, soft, solve)
            x, u, J, error, delta_J = st["x"], st["u"], st["J"], st["error"], st["delta_J"]
            if st["succeeded"]:
                drho = min(drho / o["rho_factor_SQP_DDP"], 1 / o["rho_factor_SQP_DDP"])
                rho = max(rho * drho, o["rho_min_SQP_DDP"])
            trace.append(dict(outer_iteration=outer, iteration=it, line_search_iteration=st["ls"],
                              alpha=st["alpha"], rho=rho, J=J, dV1=st["dV1"], reduction_ratio=st["ratio"],
                              succeeded_line_search=st["succeeded"]))
            exit_flag = False
            if error:
                drho = max(drho * o["rho_factor_SQP_DDP"], o["rho_factor_SQP_DDP"])
                rho = max(rho * drho, o["rho_min_SQP_DDP"])
                if rho > o["rho_max_SQP_DDP"]:
                    exit_code, exit_flag = 2, True
            elif delta_J < o["exit_tolerance_SQP_DDP"]:
                exit_code, exit_flag = 1, True
            if it == o["max_iter_SQP_DDP"] - 1:
                exit_code, exit_flag = 3, True
            else:
                it += 1
            if exit_flag:
                break
        done = False
        max_c = soft.max_value(x, u) if soft is not None else 0
        if max_c < o["exit_tolerance_softConstraints"]:
            exit_soft, done = 1, True
        if outer == o["max_iter_softConstraints"] - 1:
            exit_soft, done = 2, True
        else:
            outer += 1
        if not done and soft.update(x, u):
            exit_soft, done = 3, True
        if done:
            break
    return dict(x=x, u=u, exit_code=exit_code, exit_soft=exit_soft, outer_iter=outer, iter=it, trace=trace)
