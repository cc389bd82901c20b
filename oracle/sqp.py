"""SQP / Schur / GBD-PCG restated from the reference, blockwise.

Follows TrajoptMPCReference.py (SQP :510-760, formKKTSystemBlocks :200-271,
solveKKTSystem_Schur :415-455, reduce_regularization :457-461,
check_for_exit_or_error :463-481) and GBD-PCG-Python/PCG.py (pcg :66-111,
compute_preconditioner :166-212).  The reference forms dense G (n_xu(N-1)+nx)^2,
inverts it and multiplies dense C G^-1 C^T; S is exactly block-tridiagonal
 so we form the same blocks directly:

  Ghat_k = (G_k + rho I)^-1,  AB_k = [A_k B_k],  E = [I_nx 0]
  S_00 = -E Ghat_0 E^T
  S_{k+1,k+1} = -(AB_k Ghat_k AB_k^T + E Ghat_{k+1} E^T)
  S_{k+1,k} = AB_k Ghat_k E^T,   S_{k,k+1} = S_{k+1,k}^T
  gamma_0 = c_0 - E Ghat_0 g_0
  gamma_{k+1} = c_{k+1} + AB_k Ghat_k g_k - E Ghat_{k+1} g_{k+1}
  dxu_k = Ghat_k (g_k - (C^T lambda)_k),
  (C^T lambda)_k = [lambda_k - A_k^T lambda_{k+1}; -B_k^T lambda_{k+1}]

QuadraticCost (TrajoptCost.py:24-104), no constraints (the reference default
TrajoptConstraint(), the pinned configuration of SURVEY §0) or soft box limits
(oracle/soft.py: KKT gradient + rank-one Hessian terms, merit cost and D
terms, and the augmented-Lagrangian outer loop :483-508).
"""
import copy

import numpy as np

from . import rbd


class QuadCost:
    """QuadraticCost (TrajoptCost.py:24-104)."""

    def __init__(self, Q, QF, R, xg, QF_start=None):
        self.Q, self.QF, self.R, self.xg, self.QF_start = Q, QF, R, xg, QF_start

    def currQ(self, terminal, k):
        shifted = self.QF_start is not None and k is not None and k >= self.QF_start
        return self.QF if (terminal or shifted) else self.Q

    def value(self, x, u, k):
        dx = x - self.xg
        Qc = self.currQ(u is None, k)
        v = 0.5 * np.matmul(dx.T, np.matmul(Qc, dx))
        if u is not None:
            v += 0.5 * np.matmul(u.T, np.matmul(self.R, u))
        return v

    def gradient(self, x, u, k):
        dx = x - self.xg
        top = np.matmul(dx.T, self.currQ(u is None, k))
        return top if u is None else np.hstack((top, np.matmul(u.T, self.R)))

    def hessian(self, u_is_none, k):
        Qc = self.currQ(u_is_none, k)
        if u_is_none:
            return Qc
        nx, nu = self.Q.shape[0], self.R.shape[0]
        return np.vstack((np.hstack((Qc, np.zeros((nx, nu)))), np.hstack((np.zeros((nu, nx)), self.R))))


def default_options(options=None):
    """set_default_options (TrajoptMPCReference.py:91-115)."""
    o = {} if options is None else dict(options)
    for k, v in [("exit_tolerance_linSys", 1e-6), ("max_iter_linSys", 100), ("exit_tolerance_SQP_DDP", 1e-6),
                 ("max_iter_SQP_DDP", 100), ("alpha_factor_SQP_DDP", 0.5), ("alpha_min_SQP_DDP", 0.005),
                 ("rho_factor_SQP_DDP", 4), ("rho_min_SQP_DDP", 1e-3), ("rho_max_SQP_DDP", 1e3),
                 ("rho_init_SQP_DDP", 0.001), ("expected_reduction_min_SQP_DDP", 0.05),
                 ("expected_reduction_max_SQP_DDP", 3), ("exit_tolerance_softConstraints", 1e-6),
                 ("max_iter_softConstraints", 10)]:
        o.setdefault(k, v)
    return o


# ------------------------------------------------------------------- QP pieces
def kkt_blocks(model, cost, x, u, xs, N, dt, soft=None):
    """formKKTSystemBlocks (:200-271), returned blockwise:
    G (list of n_xu^2 / terminal nx^2), g (list), A, B (N-1), c (N, nx).
    Soft limits add their jacobian to g_k and its outer product to G_k (:220-225, :255-259)."""
    n = model.n
    nx = 2 * n
    X = x[:, :N - 1].T
    U = u.T
    A, B = rbd.euler_gradient(model, X, U, dt)
    xkp1 = rbd.euler(model, X, U, dt)
    c = np.zeros((N, nx))
    c[0] = x[:, 0] - xs
    c[1:] = x[:, 1:].T - xkp1
    if getattr(cost, "state_hessian", False):     # UrdfCost: hessian depends on x_k (TrajoptCost.py:482-519)
        G = [cost.hessian(False, k, x[:, k]) for k in range(N - 1)] + [cost.hessian(True, N - 1, x[:, N - 1])]
    else:
        G = [cost.hessian(False, k) for k in range(N - 1)] + [cost.hessian(True, N - 1)]
    g = [cost.gradient(x[:, k], u[:, k], k) for k in range(N - 1)] + [cost.gradient(x[:, N - 1], None, N - 1)]
    if soft is not None:
        nxu = nx + n
        for k in range(N):
            uk = u[:, k] if k < N - 1 else None
            js = soft.jacobians(x[:, k], uk, k, N, nxu if k < N - 1 else nx)
            if js:
                g[k] = g[k] + sum(js)
                G[k] = G[k] + sum(np.outer(j, j) for j in js)
    return G, g, A, B, c


def schur_blocks(G, g, A, B, c, rho, nx):
    N = len(G)
    Gh = [np.linalg.inv(Gk + rho * np.eye(Gk.shape[0])) for Gk in G]
    Sd = np.zeros((N, nx, nx))
    Sl = np.zeros((N - 1, nx, nx))       # S_{k+1,k}
    gam = np.zeros((N, nx))
    Sd[0] = -Gh[0][:nx, :nx]
    gam[0] = c[0] - (Gh[0] @ g[0])[:nx]
    for k in range(N - 1):
        AB = np.hstack((A[k], B[k]))
        ABG = AB @ Gh[k]
        Sd[k + 1] = -(ABG @ AB.T + Gh[k + 1][:nx, :nx])
        Sl[k] = ABG[:, :nx]
        gam[k + 1] = c[k + 1] + ABG @ g[k] - (Gh[k + 1] @ g[k + 1])[:nx]
    return Gh, Sd, Sl, gam


def dense_from_blocks(Dg, Lo, Up):
    N, b, _ = Dg.shape
    M = np.zeros((N * b, N * b))
    for k in range(N):
        M[k * b:(k + 1) * b, k * b:(k + 1) * b] = Dg[k]
    for k in range(N - 1):
        M[(k + 1) * b:(k + 2) * b, k * b:(k + 1) * b] = Lo[k]
        M[k * b:(k + 1) * b, (k + 1) * b:(k + 2) * b] = Up[k]
    return M


def preconditioner(Sd, Sl, Su, ptype):
    """compute_preconditioner, numpy branch (PCG.py:166-212), blockwise.
    Returns (P_diag, P_lo[k]=P_{k+1,k}, P_up[k]=P_{k,k+1})."""
    N, b, _ = Sd.shape
    Pl = np.zeros((N - 1, b, b))
    Pu = np.zeros((N - 1, b, b))
    if ptype == "0":   # identity (PCG.py:114-118)
        return np.array([np.eye(b) for _ in range(N)]), Pl, Pu
    if ptype == "J":
        Pd = np.array([np.linalg.inv(np.diag(np.diag(Sd[k]))) for k in range(N)])
        return Pd, Pl, Pu
    Pd = np.array([np.linalg.inv(Sd[k]) for k in range(N)])
    if ptype == "BJ":
        return Pd, Pl, Pu
    if ptype != "SS":
        raise ValueError(ptype)
    for k in range(N):
        if k % 2:     # odd row: P_{k,k-1} = -P_kk (S_{k,k-1} P_{k-1,k-1})
            Pl[k - 1] = -np.matmul(Pd[k], np.matmul(Sl[k - 1], Pd[k - 1]))
        elif k > 0:   # previous odd row: P_{k-1,k} = -P_{k-1,k-1} (S_{k-1,k} P_kk)
            Pu[k - 1] = -np.matmul(Pd[k - 1], np.matmul(Su[k - 1], Pd[k]))
    for k in range(N):
        if k % 2:
            Pu[k - 1] = Pl[k - 1].T
            if k < N - 1:
                Pl[k] = Pu[k].T
    return Pd, Pl, Pu


def block_tridiag_mv(Dg, Lo, Up, v):
    N, b, _ = Dg.shape
    V = v.reshape(N, b)
    out = np.einsum("kij,kj->ki", Dg, V)
    out[1:] += np.einsum("kij,kj->ki", Lo, V[:-1])
    out[:-1] += np.einsum("kij,kj->ki", Up, V[1:])
    return out.reshape(-1)


def pcg(Sd, Sl, Su, b, Pd, Pl, Pu, tol=1e-6, max_iter=100, guess=None):
    """PCG.pcg (PCG.py:66-111): x0 = guess (default 0, :11-12), exit on |nu'| < tol.
    Returns (x, trace_nu (abs), trace_res, iterations)."""
    def A(v):
        return block_tridiag_mv(Sd, Sl, Su, v)

    def P(v):
        return block_tridiag_mv(Pd, Pl, Pu, v)
    x = np.zeros_like(b) if guess is None else np.array(guess, dtype=float).reshape(-1)
    r = b - A(x)
    rt = P(r)
    p = rt
    nu = r @ rt
    trace = [nu]
    trace2 = [np.linalg.norm(b - A(x))]
    for _ in range(max_iter):
        Ap = A(p)
        alpha = nu / (p @ Ap)
        r = r - Ap * alpha
        x = x + p * alpha
        rt = P(r)
        nu_p = r @ rt
        trace.append(nu_p)
        trace2.append(np.linalg.norm(b - A(x)))
        if abs(nu_p) < tol:
            break
        beta = nu_p / nu
        p = rt + p * beta
        nu = nu_p
    return x, [abs(t) for t in trace], trace2, len(trace) - 1


def recover_dxu(Gh, g, A, B, lam, nx):
    N = len(Gh)
    L = lam.reshape(N, nx)
    out = []
    for k in range(N - 1):
        ctl = np.concatenate([L[k] - A[k].T @ L[k + 1], -B[k].T @ L[k + 1]])
        out.append(Gh[k] @ (g[k] - ctl))
    out.append(Gh[N - 1] @ (g[N - 1] - L[N - 1]))
    return np.concatenate(out + [lam])


def solve_qp(model, cost, x, u, xs, N, dt, rho, method, options, soft=None, guess=None):
    """One QP: returns (dxul, pcg_iters or None, extras).  guess: PCG initial iterate
    (options['guess'] of solveKKTSystem_Schur, :439-440)."""
    nx = 2 * model.n
    G, g, A, B, c = kkt_blocks(model, cost, x, u, xs, N, dt, soft)
    Gh, Sd, Sl, gam = schur_blocks(G, g, A, B, c, rho, nx)
    Su = np.transpose(Sl, (0, 2, 1))
    gamma = gam.reshape(-1)
    if method == "S":
        lam = np.linalg.solve(dense_from_blocks(Sd, Sl, Su), gamma)
        iters = None
    elif method.startswith("PCG-"):
        Pd, Pl, Pu = preconditioner(Sd, Sl, Su, method[4:])
        lam, _, _, iters = pcg(Sd, Sl, Su, gamma, Pd, Pl, Pu, options["exit_tolerance_linSys"],
                               options["max_iter_linSys"], guess)
    else:
        raise ValueError(f"oracle supports S / PCG-J / PCG-BJ / PCG-SS, got {method}")
    return recover_dxu(Gh, g, A, B, lam, nx), iters, dict(G=G, g=g, A=A, B=B, c=c, Sd=Sd, Sl=Sl, gamma=gamma,
                                                          lam=lam)


# ------------------------------------------------------------------- merit pieces
def total_cost(cost, x, u, N, soft=None):
    """totalCost (:296-310), sequential sum as the reference (soft terms after the cost terms)."""
    J = 0
    for k in range(N - 1):
        J = J + cost.value(x[:, k], u[:, k], k)
    J = J + cost.value(x[:, N - 1], None, N - 1)
    if soft is not None:
        for k in range(N - 1):
            J = J + soft.value(x[:, k], u[:, k], k, N)
        J = J + soft.value(x[:, N - 1], None, N - 1, N)
    return J


def total_violation(model, x, u, xs, N, dt, hard=None):
    """totalHardConstraintViolation (:273-294), mode sum: initial state and dynamics defects, then
    the hard box-constraint terms knot by knot (oracle/hard.py)."""
    cval = sum(map(abs, x[:, 0] - xs))
    xkp1 = rbd.euler(model, x[:, :N - 1].T, u.T, dt)
    for k in range(N - 1):
        cval = cval + sum(map(abs, x[:, k + 1] - xkp1[k]))
    if hard is not None:
        for t in hard.violation_terms(x, u, N):
            cval = cval + t
    return cval


# ------------------------------------------------------------------- SQP
def line_search(cost, model, x, u, xs, N, dt, dxul, J, merit, mu, o, soft=None, hard=None):
    """The SQP's merit line search (TrajoptMPCReference.py:640-700): trials x - alpha dx, u - alpha du
    for alpha = 1, alpha_factor, ... down to alpha_min; a trial is accepted when the merit does not
    increase and its reduction ratio lies in [expected_reduction_min, expected_reduction_max].  Returns
    the accepted (or last) trial: succeeded_line_search, alpha, ls (trials - 1), the new x, u, J, c,
    merit, D, ratio and delta_J = J - J_new."""
    nx = x.shape[0]
    n = nx + u.shape[0]
    dxul = np.asarray(dxul, dtype=float).reshape(-1, 1)
    alpha = 1
    ls = 0
    while True:
        x_new = copy.deepcopy(x)
        u_new = copy.deepcopy(u)
        for k in range(N):
            x_new[:, k] = x_new[:, k] - alpha * dxul[n * k:n * k + nx, 0]
            if k < N - 1:
                u_new[:, k] = u_new[:, k] - alpha * dxul[n * k + nx:n * (k + 1), 0]
        J_new = total_cost(cost, x_new, u_new, N, soft)
        c_new = total_violation(model, x_new, u_new, xs, N, dt, hard)
        D = 0
        for k in range(N - 1):
            D += float(cost.gradient(x_new[:, k], u_new[:, k], k) @ dxul[n * k:n * (k + 1), 0])
            if soft is not None:
                for j in soft.jacobians(x_new[:, k], u_new[:, k], k, N, n):
                    D += float(j.dot(dxul[n * k:n * (k + 1), 0]))
        D += float(cost.gradient(x_new[:, N - 1], None, N - 1) @ dxul[n * (N - 1):n * (N - 1) + nx, 0])
        if soft is not None:
            for j in soft.jacobians(x_new[:, N - 1], None, N - 1, N, nx):
                D += float(j.dot(dxul[n * (N - 1):n * (N - 1) + nx, 0]))
        merit_new = J_new + mu * c_new
        delta_J = J - J_new
        delta_merit = merit - merit_new
        with np.errstate(divide="ignore", invalid="ignore"):
            ratio = np.float64(delta_merit) / np.float64(alpha * (D - mu * c_new))
        out = dict(alpha=alpha, ls=ls, x=x_new, u=u_new, J=J_new, c=c_new, merit=merit_new, D=D, ratio=ratio,
                   delta_J=delta_J)
        if (delta_merit >= 0 and ratio >= o["expected_reduction_min_SQP_DDP"]
                and ratio <= o["expected_reduction_max_SQP_DDP"]):
            out["succeeded_line_search"] = True
            return out
        elif alpha > o["alpha_min_SQP_DDP"]:
            alpha *= o["alpha_factor_SQP_DDP"]
            ls += 1
        else:
            out["succeeded_line_search"] = False
            return out


def sqp(model, cost, x, u, N, dt, method="PCG-SS", options=None, soft=None, warm=None, hard=None,
        order="numpy"):
    """TrajoptMPCReference.SQP (:510-760).  Returns a dict.  `soft` (oracle.soft.SoftConstraints)
    enables the soft-constraint terms and the outer loop; its mu/lambda/phi are updated in place
    (the reference keeps them in the constraint object).
    `warm` (build option pcg_warm_start, include/tmpc.h): a dict whose "lam" (None = zeros) is each
    QP's PCG initial iterate and receives that QP's lambda -- the reference never forwards a guess
    from SQP (:512-519), so warm=None is the reference behaviour.
    `hard` (oracle.hard.HardConstraints): ACTIVE_SET / FULL_SET rows in the dense KKT system
    (the reference's own dense formation, small sizes only); `order` selects its PCG's summation
    order (oracle/hard.py solve_qp_dense: "numpy" the reference's, "canonical" the GPU's)."""
    o = default_options(options)
    nx, nu = 2 * model.n, model.n
    n = nx + nu
    x = np.array(x, dtype=float)
    u = np.array(u, dtype=float)
    xs = copy.deepcopy(x[:, 0])
    outer = 0
    exit_soft = 0
    while True:
        rho = o["rho_init_SQP_DDP"]
        drho = 1
        J = total_cost(cost, x, u, N, soft)
        c = total_violation(model, x, u, xs, N, dt, hard)
        mu = 10
        merit = J + mu * c
        trace = [dict(outer_iteration=outer, iteration=0, line_search_iteration=0, alpha=1, rho=rho, J=J, c=c,
                      merit=merit, D=None, reduction_ratio=None, succeeded_line_search=False)]
        pcg_iters, dxuls, active_rows, active_sets, active_masks, singular, iterates = [], [], [], [], [], [], []
        it = 0
        exit_sqp = 0
        while True:
            iterates.append((x.copy(), u.copy(), rho))
            if hard is not None or method == "N":
                from . import hard as ohard
                hc = hard if hard is not None else ohard.HardConstraints([])
                G, g, C, cc = ohard.kkt_dense(model, cost, x, u, xs, N, dt, hc, soft)
                if method == "N":   # solveKKTSystem (:313-359), the reference's default method
                    dxul, sing = ohard.solve_kkt_dense(G, g, C, cc, rho)
                    iters = None
                else:
                    fl = {}
                    dxul, iters, _ = ohard.solve_qp_dense(G, g, C, cc, rho, method, o, nx, fl, order)
                    sing = fl.get("singular", False)
                singular.append(bool(sing))
                active_rows.append(C.shape[0] - nx * N)
                active_sets.append([(k, int(sg)) for k in range(N)
                                    for _, sg, _ in hc.rows(x[:, k], u[:, k] if k < N - 1 else None, k, N)])
                active_masks.append(hc.active_masks(x, u, N))
            else:
                singular.append(False)
                guess = None if warm is None else warm.get("lam")
                dxul, iters, ex = solve_qp(model, cost, x, u, xs, N, dt, rho, method, o, soft, guess)
                if warm is not None and iters is not None:
                    warm["lam"] = ex["lam"].copy()
            dxul = dxul.reshape(-1, 1)
            dxuls.append(dxul[:, 0].copy())
            if iters is not None:
                pcg_iters.append(iters)
            r = line_search(cost, model, x, u, xs, N, dt, dxul, J, merit, mu, o, soft, hard)
            error = not r["succeeded_line_search"]
            if not error:
                x, u, J, c, merit = r["x"], r["u"], r["J"], r["c"], r["merit"]
                drho = min(drho / o["rho_factor_SQP_DDP"], 1 / o["rho_factor_SQP_DDP"])
                rho = max(rho * drho, o["rho_min_SQP_DDP"])
            delta_J = r["delta_J"]
            trace.append(dict(outer_iteration=outer, iteration=it, line_search_iteration=r["ls"], alpha=r["alpha"],
                              rho=rho, J=J, c=c, merit=merit, D=r["D"], reduction_ratio=r["ratio"],
                              succeeded_line_search=not error))
            # check_for_exit_or_error (:463-481)
            exit_flag = False
            if error:
                drho = max(drho * o["rho_factor_SQP_DDP"], o["rho_factor_SQP_DDP"])
                rho = max(rho * drho, o["rho_min_SQP_DDP"])
                if rho > o["rho_max_SQP_DDP"]:
                    exit_sqp, exit_flag = 2, True
            elif delta_J < o["exit_tolerance_SQP_DDP"]:
                exit_sqp, exit_flag = 1, True
            if it == o["max_iter_SQP_DDP"] - 1:
                exit_sqp, exit_flag = 3, True
            else:
                it += 1
            if exit_flag:
                break
        # check_and_update_soft_constraints (:483-508); without soft limits the max value is 0 < tol
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
    return dict(x=x, u=u, exit_sqp=exit_sqp, exit_soft=exit_soft, outer_iter=outer, sqp_iter=it, trace=trace,
                pcg_iters=pcg_iters, dxul=dxuls, active_rows=active_rows, active_sets=active_sets,
                active_masks=active_masks, singular=singular, iterates=iterates)


def initial_problem(model, N, dt, seed):
    """§8d workload: q0 ~ U(-1,1)^n (default_rng(seed)), qd0 = 0, Euler rollout of u = 0."""
    n = model.n
    rng = np.random.default_rng(seed)
    x = np.zeros((2 * n, N))
    x[:n, 0] = rng.uniform(-1.0, 1.0, n)
    u = np.zeros((n, N - 1))
    for k in range(N - 1):
        x[:, k + 1] = rbd.euler(model, x[:, k][None], u[:, k][None], dt)[0]
    return x, u
