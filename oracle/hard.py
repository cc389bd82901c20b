"""Hard box constraints (BoxConstraint modes ACTIVE_SET / FULL_SET).  TEST
INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates, densely and in the reference's own row order:
  * TrajoptConstraint.value_hard_constraints / jacobian_hard_constraints
    (TrajoptConstraint.py:53-128, 210-274): per knot, joint then velocity then
    torque limits; full value [z - lb; ub - z]; ACTIVE_SET keeps the entries < 0
    (and the jacobian rows that are not all zero, +1 for a lower, -1 for an
    upper bound), FULL_SET keeps all of them (an inactive row's jacobian is 0);
    torque limits have no terminal-knot rows (:230);
  * formKKTSystemBlocks' hard rows (TrajoptMPCReference.py:238-248, 262-270):
    appended to C / c right after each knot's dynamics rows;
  * totalHardConstraintViolation's hard terms (:286-293), summed after the
    dynamics defects, knot by knot;
  * solveKKTSystem_Schur on the dense system (:415-455) and GBD-PCG's
    compute_preconditioner on nx-aligned blocks of the dense S (PCG.py:113-212):
    n_blocks = floor(dim / nx), so with hard rows the blocks no longer line up
    with the knots and the trailing dim mod nx rows are not preconditioned.

Semantics for constraint_size > 1 (the reference cannot run them):
the elementwise generalisation -- full value concatenated [z - lb; ub - z] (2 cs
entries, lower bounds first), one row per selected entry with a single +-1 in
its column.  The reference's terminal hard rows for joint / velocity limits are
reshaped to nx columns (:269) and crash for constraint_size 1 (a 2-row, 3-column
jacobian); here they keep their state columns.
"""
import numpy as np

KINDS = ("joint", "velocity", "torque")
MODES = ("ACTIVE_SET", "FULL_SET")


class HardLimit:
    def __init__(self, kind, n, lb, ub, mode):
        if kind not in KINDS or mode not in MODES:
            raise ValueError((kind, mode))
        self.kind, self.n, self.mode = kind, n, mode
        self.lb = np.broadcast_to(np.asarray(lb, dtype=float), (n,)).copy()
        self.ub = np.broadcast_to(np.asarray(ub, dtype=float), (n,)).copy()

    def col0(self):
        """first column of the limited slice in a knot's [q; qd; u] block"""
        return KINDS.index(self.kind) * self.n


class HardConstraints:
    def __init__(self, limits):
        self.limits = [lim for k in KINDS for lim in limits if lim.kind == k]   # reference order

    def rows(self, xk, uk, k, N):
        """[(column in [x_k; u_k], sign, value)] of knot k, in the reference's row order."""
        out = []
        for lim in self.limits:
            if lim.kind == "torque" and (k >= N - 1 or uk is None):
                continue
            n = lim.n
            z = uk if lim.kind == "torque" else xk[lim.col0():lim.col0() + n]
            full = np.concatenate([z - lim.lb, lim.ub - z])
            for e in range(2 * n):
                active = full[e] < 0
                if lim.mode == "ACTIVE_SET" and not active:
                    continue
                sign = (1.0 if e < n else -1.0) if active else 0.0
                out.append((lim.col0() + (e % n), sign, full[e]))
        return out

    def violation_terms(self, x, u, N):
        """the per-knot sum(map(abs, c_err)) terms of :286-293, in order"""
        terms = []
        for k in range(N):
            r = self.rows(x[:, k], u[:, k] if k < N - 1 else None, k, N)
            if r:
                terms.append(sum(map(abs, [v for _, _, v in r])))
        return terms


def kkt_dense(model, cost, x, u, xs, N, dt, hard, soft=None):
    """formKKTSystemBlocks, numpy branch (:200-271): dense G, g, C, c with the hard rows."""
    from . import rbd
    n = model.n
    nx, nu = 2 * n, n
    nxu = nx + nu
    X = x[:, :N - 1].T
    U = u.T
    A, B = rbd.euler_gradient(model, X, U, dt)
    xkp1 = rbd.euler(model, X, U, dt)
    nz = nxu * (N - 1) + nx
    Crows, crow = [], []
    G = np.zeros((nz, nz))
    g = np.zeros(nz)
    row = np.zeros(nz)
    row[:nx] = 0
    for i in range(nx):
        r = np.zeros(nz)
        r[i] = 1.0
        Crows.append(r)
        crow.append(x[i, 0] - xs[i])
    for k in range(N - 1):
        s = k * nxu
        G[s:s + nxu, s:s + nxu] = cost.hessian(False, k)
        g[s:s + nxu] = cost.gradient(x[:, k], u[:, k], k)
        if soft is not None:
            for j in soft.jacobians(x[:, k], u[:, k], k, N, nxu):
                g[s:s + nxu] += j
                G[s:s + nxu, s:s + nxu] += np.outer(j, j)
        for i in range(nx):
            r = np.zeros(nz)
            r[s:s + nx] = -A[k][i]
            r[s + nx:s + nxu] = -B[k][i]
            r[s + nxu + i] = 1.0
            Crows.append(r)
            crow.append(x[i, k + 1] - xkp1[k][i])
        for col, sign, val in hard.rows(x[:, k], u[:, k], k, N):
            r = np.zeros(nz)
            r[s + col] = sign
            Crows.append(r)
            crow.append(val)
    s = (N - 1) * nxu
    G[s:, s:] = cost.hessian(True, N - 1)
    g[s:] = cost.gradient(x[:, N - 1], None, N - 1)
    if soft is not None:
        for j in soft.jacobians(x[:, N - 1], None, N - 1, N, nx):
            g[s:] += j
            G[s:, s:] += np.outer(j, j)
    for col, sign, val in hard.rows(x[:, N - 1], None, N - 1, N):
        r = np.zeros(nz)
        r[s + col] = sign
        Crows.append(r)
        crow.append(val)
    return G, g, np.array(Crows), np.array(crow)


def preconditioner_dense(S, nx, ptype):
    """compute_preconditioner, numpy branch (PCG.py:113-212), on the dense S."""
    dim = S.shape[0]
    if ptype == "0":
        return np.identity(dim)
    if ptype == "J":
        return np.linalg.inv(np.diag(np.diag(S)))
    nb = int(dim / nx)
    P = np.zeros(S.shape)
    for k in range(nb):
        P[k * nx:(k + 1) * nx, k * nx:(k + 1) * nx] = np.linalg.inv(S[k * nx:(k + 1) * nx, k * nx:(k + 1) * nx])
        if ptype != "SS":
            continue
        if k % 2:
            P[k * nx:(k + 1) * nx, (k - 1) * nx:k * nx] = -np.matmul(
                P[k * nx:(k + 1) * nx, k * nx:(k + 1) * nx],
                np.matmul(S[k * nx:(k + 1) * nx, (k - 1) * nx:k * nx], P[(k - 1) * nx:k * nx, (k - 1) * nx:k * nx]))
        elif k > 0:
            P[(k - 1) * nx:k * nx, k * nx:(k + 1) * nx] = -np.matmul(
                P[(k - 1) * nx:k * nx, (k - 1) * nx:k * nx],
                np.matmul(S[(k - 1) * nx:k * nx, k * nx:(k + 1) * nx], P[k * nx:(k + 1) * nx, k * nx:(k + 1) * nx]))
    if ptype == "SS":
        for k in range(nb):
            if k % 2:
                P[(k - 1) * nx:k * nx, k * nx:(k + 1) * nx] = P[k * nx:(k + 1) * nx, (k - 1) * nx:k * nx].T
                if k < nb - 1:
                    P[(k + 1) * nx:(k + 2) * nx, k * nx:(k + 1) * nx] = P[k * nx:(k + 1) * nx, (k + 1) * nx:(k + 2) * nx].T
    return P


def pcg_dense(S, b, P, tol, max_iter):
    """PCG.pcg (PCG.py:66-111) with x0 = 0."""
    x = np.zeros_like(b)
    r = b - S @ x
    rt = P @ r
    p = rt
    nu = r @ rt
    it = 0
    for it in range(1, max_iter + 1):
        Ap = S @ p
        alpha = nu / (p @ Ap)
        r = r - Ap * alpha
        x = x + p * alpha
        rt = P @ r
        nup = r @ rt
        if abs(nup) < tol:
            break
        beta = nup / nu
        p = rt + p * beta
        nu = nup
    return x, it


def solve_qp_dense(G, g, C, c, rho, method, options, nx):
    """solveKKTSystem_Schur, numpy branch (:415-455).  Method S uses np.linalg.solve; when S is
    singular (FULL_SET: the inactive rows of C are zero) the reference falls back to lstsq (:431-436)."""
    Gr = G + rho * np.eye(G.shape[0])
    invG = np.linalg.inv(Gr)
    S = -np.matmul(C, np.matmul(invG, C.T))
    gamma = c - np.matmul(C, np.matmul(invG, g))
    iters = None
    if method == "S":
        try:
            lam = np.linalg.solve(S, gamma)
        except np.linalg.LinAlgError:
            lam = np.linalg.lstsq(S, gamma, rcond=None)[0]
    else:
        P = preconditioner_dense(S, nx, method[4:])
        lam, iters = pcg_dense(S, gamma, P, options["exit_tolerance_linSys"], options["max_iter_linSys"])
    dxu = invG @ (g - C.T @ lam)
    return np.concatenate([dxu, lam]), iters, S
