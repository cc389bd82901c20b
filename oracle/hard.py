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

    def active_masks(self, x, u, N):
        """Per knot, the active-set bitmask of the QP's hard rows: bit t * 2n + e for limit kind t
        (0 joint, 1 velocity, 2 torque) and entry e of [z - lb; ub - z] (e < n lower bound, e >= n
        upper), set when that entry is violated (< 0) -- ACTIVE_SET's rows, FULL_SET's nonzero rows.
        The GPU reports the same masks (tmpc_trace.hard_active, tmpc_qp_hard_info)."""
        out = []
        for k in range(N):
            m = 0
            for col, sign, _ in self.rows(x[:, k], u[:, k] if k < N - 1 else None, k, N):
                if sign == 0:
                    continue
                n = self.limits[0].n if self.limits else 1
                t, i = divmod(col, n)
                m |= 1 << (t * 2 * n + (i if sign > 0 else n + i))
            out.append(m)
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


# ------------------------------------------------------------------ canonical summation order
# PCG on these active-set Schur complements (the trailing dim mod nx rows have no preconditioner
# rows, PCG.py:182) is summation-order sensitive: on the SAME S, the reference's NumPy / OpenBLAS
# order (pcg_dense with preconditioner_dense, CPU-dependent) and a plain sequential order
# stop up to 5 iterations apart on the arm3 cases of tests/test_gpu_hard.py.  So the oracle fixes
# ONE order -- every sum sequential from 0.0 in index order, every product and sum rounded on its
# own (no fused multiply-add), dot products as per-thread partials over PCG_THREADS = 1024 threads
# (row a on thread a mod 1024) reduced by a 64-lane xor butterfly and a fan-in over the 16 waves -- and the GPU's
# k_hard_pcg follows it operation for operation (tmpc_hard.hip, fp contraction off), so the two are
# bitwise equal on identical S and gamma.  The reference's own fixtures pin both orders on their
# integers except where a count is decided by the order itself: the pendulum ACTIVE_SET PCG-SS run's
# QPs 2 and 6 stop one iteration apart (42 vs 41 at QP 2, 7 active rows)
# (tests/test_oracle_golden.py::test_canonical_order_on_reference_fixtures).

def _gj_inverse(M):
    """Gauss-Jordan inverse of the augmented [M | I] without pivoting (principal blocks of the
    negative definite S), in place of np.linalg.inv's LU: row p /= pivot, then every other row r
    -= M[r, p] * row p."""
    M = np.array(M, dtype=float)
    n = M.shape[0]
    for p in range(n):
        d = M[p, p]
        row = M[p] / d
        row[p] = 1.0 / d
        M[p] = row
        for r in range(n):
            if r == p:
                continue
            f = M[r, p]
            M[r, p] = 0.0
            M[r] = M[r] - f * M[p]
    return M


def _neg_triple(X, Y, Z):
    """-(X (Y Z)), both products summed sequentially (PCG.py:196-206's -P (S P))."""
    n = X.shape[0]
    yz = np.zeros((n, n))
    for l in range(n):
        yz = yz + Y[:, l:l + 1] * Z[l:l + 1, :]
    acc = np.zeros((n, n))
    for m in range(n):
        acc = acc + X[:, m:m + 1] * yz[m:m + 1, :]
    return -acc


PCG_THREADS = 1024   # k_hard_pcg's workgroup (tmpc_internal.h HARD_PCG_THREADS)


def _dot(a, b):
    """sum(a * b): per-thread partials (thread t sums rows t, t + 1024, ... in order), a 64-lane xor
    butterfly per wave, then the 16 wave totals in order."""
    T = PCG_THREADS
    prod = a * b
    D = len(prod)
    J = (D + T - 1) // T
    pad = np.zeros(J * T)
    pad[:D] = prod
    part = np.zeros(T)
    for j in range(J):
        part = part + pad[j * T:(j + 1) * T]
    idx = np.arange(T)
    for off in (32, 16, 8, 4, 2, 1):
        part = part + part[idx ^ off]
    s = 0.0
    for w in range(T // 64):
        s = s + part[w * 64]
    return s


def preconditioner_canonical(S, nx, ptype):
    """compute_preconditioner (PCG.py:113-212) in the canonical order: the diagonal blocks of the
    first floor(dim / nx) nx-aligned blocks by _gj_inverse, SS's stair blocks P_{k,k-1} = -P_kk
    (S_{k,k-1} P_{k-1,k-1}) for odd k and P_{k-1,k} = -P_{k-1,k-1} (S_{k-1,k} P_kk) for even k, each
    mirrored by its transpose.  Returns (Pd [nb][nx][nx], Pl [nb-1][nx][nx] = P_{k+1,k})."""
    nb = S.shape[0] // nx
    Pd = np.zeros((nb, nx, nx))
    Pl = np.zeros((max(nb - 1, 0), nx, nx))
    if ptype in ("BJ", "SS"):
        for k in range(nb):
            Pd[k] = _gj_inverse(S[k * nx:(k + 1) * nx, k * nx:(k + 1) * nx])
    if ptype == "SS":
        for k in range(1, nb):
            if k % 2:
                Pl[k - 1] = _neg_triple(Pd[k], S[k * nx:(k + 1) * nx, (k - 1) * nx:k * nx], Pd[k - 1])
            else:
                Pl[k - 1] = _neg_triple(Pd[k - 1], S[(k - 1) * nx:k * nx, k * nx:(k + 1) * nx], Pd[k]).T
    return Pd, Pl


def pcg_canonical(S, b, nx, ptype, tol, max_iter):
    """PCG.pcg (PCG.py:66-111, x0 = 0) with the preconditioner ptype in {0, J, BJ, SS} on the dense S,
    every operation in the canonical order above.  Returns (x, iterations)."""
    S = np.asarray(S, dtype=float)
    D = S.shape[0]
    nb = D // nx
    Pd, Pl = preconditioner_canonical(S, nx, ptype)
    diag = np.diag(S).copy()

    def apply_P(r):
        if ptype == "0":
            return r.copy()
        if ptype == "J":
            return (1.0 / diag) * r
        z = np.zeros(D)
        R = r[:nb * nx].reshape(nb, nx)
        s = np.zeros((nb, nx))
        for j in range(nx):
            s = s + Pd[:, :, j] * R[:, j:j + 1]
        if ptype == "SS" and nb > 1:
            for j in range(nx):       # P_{k,k-1} r_{k-1}
                s[1:] = s[1:] + Pl[:, :, j] * R[:-1, j:j + 1]
            for j in range(nx):       # P_{k,k+1} r_{k+1} = P_{k+1,k}^T r_{k+1}
                s[:-1] = s[:-1] + Pl[:, j, :] * R[1:, j:j + 1]
        z[:nb * nx] = s.reshape(-1)   # rows past the last full block: 0 (PCG.py:182)
        return z

    def spmv(v):
        s = np.zeros(D)
        for c in range(D):
            s = s + S[:, c] * v[c]
        return s

    x = np.zeros(D)
    r = np.array(b, dtype=float)
    z = apply_P(r)
    p = z.copy()
    nu = _dot(r, z)
    it_done = max_iter
    for it in range(max_iter):
        Ap = spmv(p)
        alpha = nu / _dot(p, Ap)
        r = r - Ap * alpha
        x = x + p * alpha
        z = apply_P(r)
        nup = _dot(r, z)
        if abs(nup) < tol:
            it_done = it + 1
            break
        beta = nup / nu
        p = z + p * beta
        nu = nup
    return x, it_done


def pcg_dense(S, b, P, tol, max_iter):
    """PCG.pcg (PCG.py:66-111) with x0 = 0, NumPy's summation order (the reference's own arithmetic,
    CPU-dependent; kept to document the order sensitivity, see above)."""
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


def structurally_singular(C):
    """C has a zero row (FULL_SET's inactive entries) or two rows equal up to sign (a knot-0 hard row on
    a state entry duplicates the initial-state row: xs violates a joint / velocity limit), so S = -C G^-1
    C^T is singular in exact arithmetic.  The reference's np.linalg.solve raises for the first and, for
    the second, raises or returns a rounding-sized pivot's answer depending on the elimination's
    rounding; the build defines both as singular and takes lstsq's minimum-norm answer (the
    reference's fallback, TrajoptMPCReference.py:431-436), as tmpc_hard.hip's k_hard_direct does."""
    if np.any(np.all(C == 0, axis=1)):
        return True
    seen = set()
    for row in C:
        lead = row[np.flatnonzero(row)[0]]
        key = ((row if lead > 0 else -row) + 0.0).tobytes()   # rows equal up to sign share a key (+0.0: no -0)
        if key in seen:
            return True
        seen.add(key)
    return False


def solve_kkt_dense(G, g, C, c, rho):
    """solveKKTSystem, numpy branch (TrajoptMPCReference.py:313-359): G + rho I (when rho != 0) and
    [G C^T; C 0] [dxu; lambda] = [g; c] by np.linalg.solve, falling back to lstsq with the
    `singular` flag when LAPACK reports a singular matrix (:353-357).  Returns (dxul, singular)."""
    Gr = G + rho * np.eye(G.shape[0]) if rho != 0 else G
    m = C.shape[0]
    KKT = np.hstack((np.vstack((Gr, C)), np.vstack((C.T, np.zeros((m, m))))))
    rhs = np.concatenate([g, c])
    try:
        if structurally_singular(C):   # singular KKT matrix: defined as the lstsq answer (see above)
            raise np.linalg.LinAlgError("structurally singular KKT matrix")
        return np.linalg.solve(KKT, rhs), False
    except np.linalg.LinAlgError:
        return np.linalg.lstsq(KKT, rhs, rcond=None)[0], True


def solve_qp_dense(G, g, C, c, rho, method, options, nx, flags=None, order="numpy"):
    """`flags` (a dict, optional) receives "singular": the least-squares fallback ran.  order:
    "numpy" -- the reference's own arithmetic (preconditioner_dense + pcg_dense), which reproduces
    its fixtures; "canonical" -- pcg_canonical, the order the GPU's k_hard_pcg follows bit for bit."""
    """solveKKTSystem_Schur, numpy branch (:415-455).  Method S uses np.linalg.solve; when S is
    singular (FULL_SET: the inactive rows of C are zero) the reference falls back to lstsq (:431-436)."""
    Gr = G + rho * np.eye(G.shape[0])
    invG = np.linalg.inv(Gr)
    S = -np.matmul(C, np.matmul(invG, C.T))
    gamma = c - np.matmul(C, np.matmul(invG, g))
    iters = None
    if method == "S":
        try:
            if structurally_singular(C):
                raise np.linalg.LinAlgError("structurally singular S")
            lam = np.linalg.solve(S, gamma)
        except np.linalg.LinAlgError:
            lam = np.linalg.lstsq(S, gamma, rcond=None)[0]
            if flags is not None:
                flags["singular"] = True
    else:
        ptype = method[4:]
        tol, mi = options["exit_tolerance_linSys"], options["max_iter_linSys"]
        if order == "canonical":
            if ptype in ("BJ", "SS"):   # the reference's np.linalg.inv raises on a singular block (FULL_SET)
                for k in range(S.shape[0] // nx):
                    np.linalg.inv(S[k * nx:(k + 1) * nx, k * nx:(k + 1) * nx])
            lam, iters = pcg_canonical(S, gamma, nx, ptype, tol, mi)
        else:
            lam, iters = pcg_dense(S, gamma, preconditioner_dense(S, nx, ptype), tol, mi)
    dxu = invG @ (g - C.T @ lam)
    return np.concatenate([dxu, lam]), iters, S
