"""Rigid-body dynamics restated from GRiD/RBDReference/RBDReference.py,
batched over a leading axis K (independent evaluations, e.g. knots).

Model input: a RobotModel (trajoptmpcreference_amd.urdf), whose arrays are
checked against the reference's own parser output in
tests/test_model.py (golden model_*.npz).

Shapes: q, qd, qdd, u: (K, n); spatial vectors (K, 6); matrices (K, 6, 6).
"""
import numpy as np


def xmat(model, j, q):
    """X_j(q) for a batch of q (K,) -> (K,6,6)  (Joint.py:88-100 semantics)."""
    if model.jtype[j] == 0:
        return (model.X0[j][None] + np.cos(q)[:, None, None] * model.Xa[j][None]
                + np.sin(q)[:, None, None] * model.Xb[j][None])
    return model.X0[j][None] + q[:, None, None] * model.Xa[j][None]


def _mv(M, v):
    return np.einsum("kij,kj->ki", M, v)


def _mtv(M, v):
    return np.einsum("kji,kj->ki", M, v)


def cross_operator(v):
    """crm(v)  (RBDReference.py:13-35)."""
    K = v.shape[0]
    z = np.zeros(K)
    return np.stack([
        np.stack([z, -v[:, 2], v[:, 1], z, z, z], 1),
        np.stack([v[:, 2], z, -v[:, 0], z, z, z], 1),
        np.stack([-v[:, 1], v[:, 0], z, z, z, z], 1),
        np.stack([z, -v[:, 5], v[:, 4], z, -v[:, 2], v[:, 1]], 1),
        np.stack([v[:, 5], z, -v[:, 3], v[:, 2], z, -v[:, 0]], 1),
        np.stack([-v[:, 4], v[:, 3], z, -v[:, 1], v[:, 0], z], 1)], 1)


def mxS(S, vec, alpha=None):
    """alpha * crm(vec) @ S  (RBDReference.py:57-62)."""
    r = _mv(cross_operator(vec), np.broadcast_to(S, vec.shape))
    return r if alpha is None else alpha[:, None] * r


def fxv(f, t):
    """Fx(f) * t  (RBDReference.py:71-91)."""
    r = np.empty_like(f)
    r[:, 0] = -f[:, 2] * t[:, 1] + f[:, 1] * t[:, 2] - f[:, 5] * t[:, 4] + f[:, 4] * t[:, 5]
    r[:, 1] = f[:, 2] * t[:, 0] - f[:, 0] * t[:, 2] + f[:, 5] * t[:, 3] - f[:, 3] * t[:, 5]
    r[:, 2] = -f[:, 1] * t[:, 0] + f[:, 0] * t[:, 1] - f[:, 4] * t[:, 3] + f[:, 3] * t[:, 4]
    r[:, 3] = -f[:, 2] * t[:, 4] + f[:, 1] * t[:, 5]
    r[:, 4] = f[:, 2] * t[:, 3] - f[:, 0] * t[:, 5]
    r[:, 5] = -f[:, 1] * t[:, 3] + f[:, 0] * t[:, 4]
    return r


def vxIv(v, I):
    """v x* (I v)  (RBDReference.py:98-116)."""
    t = np.einsum("ij,kj->ki", I, v)
    r = np.empty_like(v)
    r[:, 0] = -v[:, 2] * t[:, 1] + v[:, 1] * t[:, 2] + -v[:, 5] * t[:, 4] + v[:, 4] * t[:, 5]
    r[:, 1] = v[:, 2] * t[:, 0] + -v[:, 0] * t[:, 2] + v[:, 5] * t[:, 3] + -v[:, 3] * t[:, 5]
    r[:, 2] = -v[:, 1] * t[:, 0] + v[:, 0] * t[:, 1] + -v[:, 4] * t[:, 3] + v[:, 3] * t[:, 4]
    r[:, 3] = -v[:, 2] * t[:, 4] + v[:, 1] * t[:, 5]
    r[:, 4] = v[:, 2] * t[:, 3] + -v[:, 0] * t[:, 5]
    r[:, 5] = -v[:, 1] * t[:, 3] + v[:, 0] * t[:, 4]
    return r


def rnea(model, q, qd, qdd=None, gravity=-9.81):
    """rnea_fpass + rnea_bpass (RBDReference.py:399-559).  Returns (c, v, a, f)
    with f *after* the backward accumulation, as the reference returns it."""
    K, n = q.shape
    v = np.zeros((n, K, 6))
    a = np.zeros((n, K, 6))
    f = np.zeros((n, K, 6))
    g = np.zeros((K, 6))
    g[:, 5] = -gravity
    X = [xmat(model, j, q[:, j]) for j in range(n)]
    for j in range(n):
        p = model.parent[j]
        S = model.S[j]
        if p == -1:
            a[j] = _mv(X[j], g)
        else:
            v[j] = _mv(X[j], v[p])
            a[j] = _mv(X[j], a[p])
        v[j] = v[j] + S[None] * qd[:, j:j + 1]
        a[j] = a[j] + mxS(S, v[j], qd[:, j])
        if qdd is not None:
            a[j] = a[j] + S[None] * qdd[:, j:j + 1]
        f[j] = np.einsum("ij,kj->ki", model.I[j], a[j]) + vxIv(v[j], model.I[j])
    c = np.zeros((K, n))
    for j in range(n - 1, -1, -1):
        c[:, j] = f[j] @ model.S[j]
        p = model.parent[j]
        if p != -1:
            f[p] = f[p] + _mtv(X[j], f[j])
    return c, v, a, f


def rnea_grad(model, q, qd, qdd, gravity=-9.81):
    """rnea_grad (RBDReference.py:561-802) -> dc_du (K, n, 2n) = [dc/dq, dc/dqd]."""
    K, n = q.shape
    c, v, a, f = rnea(model, q, qd, qdd, gravity)
    X = [xmat(model, j, q[:, j]) for j in range(n)]
    I = model.I
    g = np.zeros((K, 6))
    g[:, 5] = -gravity
    # forward pass dq  (:561-633)
    dv = np.zeros((n, n, K, 6))     # [ind][col]
    da = np.zeros((n, n, K, 6))
    df = np.zeros((n, n, K, 6))
    for j in range(n):
        p = model.parent[j]
        S = model.S[j]
        if p != -1:
            for col in range(n):
                dv[j, col] = _mv(X[j], dv[p, col])
            dv[j, j] = dv[j, j] + mxS(S, _mv(X[j], v[p]))
            for col in range(n):
                da[j, col] = _mv(X[j], da[p, col])
        for col in range(n):
            da[j, col] = da[j, col] + mxS(S, dv[j, col], qd[:, j])
        if p != -1:
            da[j, j] = da[j, j] + mxS(S, _mv(X[j], a[p]))
        else:
            da[j, j] = da[j, j] + mxS(S, _mv(X[j], g))
        Iv = np.einsum("ij,kj->ki", I[j], v[j])
        for col in range(n):
            df[j, col] = np.einsum("ij,kj->ki", I[j], da[j, col])
            df[j, col] = df[j, col] + fxv(dv[j, col], Iv)
            df[j, col] = df[j, col] + fxv(v[j], np.einsum("ij,kj->ki", I[j], dv[j, col]))
    # forward pass dqd  (:635-690)
    dvd = np.zeros((n, n, K, 6))
    dad = np.zeros((n, n, K, 6))
    dfd = np.zeros((n, n, K, 6))
    for j in range(n):
        p = model.parent[j]
        S = model.S[j]
        if p != -1:
            for col in range(n):
                dvd[j, col] = _mv(X[j], dvd[p, col])
        dvd[j, j] = dvd[j, j] + S[None]
        if p != -1:
            for col in range(n):
                dad[j, col] = _mv(X[j], dad[p, col])
        for col in range(n):
            dad[j, col] = dad[j, col] + mxS(S, dvd[j, col], qd[:, j])
        dad[j, j] = dad[j, j] + mxS(S, v[j])
        Iv = np.einsum("ij,kj->ki", I[j], v[j])
        for col in range(n):
            dfd[j, col] = np.einsum("ij,kj->ki", I[j], dad[j, col])
            dfd[j, col] = dfd[j, col] + fxv(dvd[j, col], Iv)
            dfd[j, col] = dfd[j, col] + fxv(v[j], np.einsum("ij,kj->ki", I[j], dvd[j, col]))
    # backward pass dq  (:692-735)
    dc_dq = np.zeros((K, n, n))
    for j in range(n - 1, -1, -1):
        S = model.S[j]
        for col in range(n):
            dc_dq[:, j, col] = df[j, col] @ S
        p = model.parent[j]
        if p != -1:
            for col in range(n):
                df[p, col] = df[p, col] + _mtv(X[j], df[j, col])
            delta = _mtv(X[j], -mxS(S, f[j]))
            df[p, j] = df[p, j] + delta
    # backward pass dqd  (:737-771)
    dc_dqd = np.zeros((K, n, n))
    for j in range(n - 1, -1, -1):
        S = model.S[j]
        for col in range(n):
            dc_dqd[:, j, col] = dfd[j, col] @ S
        p = model.parent[j]
        if p != -1:
            for col in range(n):
                dfd[p, col] = dfd[p, col] + _mtv(X[j], dfd[j, col])
    return np.concatenate([dc_dq, dc_dqd], axis=2)


def minv(model, q):
    """Analytic M^-1 (RBDReference.py:805-930), symmetrised from the upper triangle."""
    K, n = q.shape
    X = [xmat(model, j, q[:, j]) for j in range(n)]
    Minv = np.zeros((K, n, n))
    F = np.zeros((n, K, 6, n))
    U = np.zeros((n, K, 6))
    Dinv = np.zeros((n, K))
    IA = [np.broadcast_to(model.I[j], (K, 6, 6)).copy() for j in range(n)]
    for j in range(n - 1, -1, -1):
        S = model.S[j]
        sub = model.subtree[j]
        U[j] = IA[j] @ S
        Dinv[j] = 1.0 / (U[j] @ S)
        Minv[:, j, j] = Dinv[j]
        for s in sub:
            Minv[:, j, s] = Minv[:, j, s] - Dinv[j] * (F[j][:, :, s] @ S)
        p = model.parent[j]
        if p != -1:
            for s in sub:
                F[j][:, :, s] = F[j][:, :, s] + U[j] * Minv[:, j, s][:, None]
                F[p][:, :, s] = F[p][:, :, s] + _mtv(X[j], F[j][:, :, s])
            Ia = IA[j] - np.einsum("ki,kj->kij", U[j], Dinv[j][:, None] * U[j])
            IA[p] = IA[p] + np.einsum("kji,kjl,klm->kim", X[j], Ia, X[j])
    for j in range(n):
        p = model.parent[j]
        S = model.S[j]
        if p != -1:
            UX = np.einsum("ki,kij->kj", U[j], X[j])
            Minv[:, j, j:] = Minv[:, j, j:] - Dinv[j][:, None] * np.einsum("ki,kis->ks", UX, F[p][:, :, j:])
        F[j][:, :, j:] = S[None, :, None] * Minv[:, j, j:][:, None, :]
        if p != -1:
            F[j][:, :, j:] = F[j][:, :, j:] + np.einsum("kij,kjs->kis", X[j], F[p][:, :, j:])
    for col in range(n):
        for row in range(n):
            if col < row:
                Minv[:, row, col] = Minv[:, col, row]
    return Minv


def forward_dynamics(model, x, u, gravity=-9.81):
    """URDFPlant.forward_dynamics (TrajoptPlant.py:283-299)."""
    n = model.n
    q, qd = x[:, :n], x[:, n:]
    c, _, _, _ = rnea(model, q, qd, None, gravity)
    Mi = minv(model, q)
    return np.einsum("kij,kj->ki", Mi, u - c)


def forward_dynamics_gradient(model, x, u, gravity=-9.81):
    """URDFPlant.forward_dynamics_gradient (TrajoptPlant.py:301-323) -> (K, n, 3n)."""
    n = model.n
    q, qd = x[:, :n], x[:, n:]
    c, _, _, _ = rnea(model, q, qd, None, gravity)
    Mi = minv(model, q)
    qdd = np.einsum("kij,kj->ki", Mi, u - c)
    dc = rnea_grad(model, q, qd, qdd, gravity)
    return np.concatenate([np.matmul(-Mi, dc), Mi], axis=2)


def euler(model, x, u, dt, gravity=-9.81):
    """TrajoptPlant.integrator type 0, no gradient (TrajoptPlant.py:92-99)."""
    n = model.n
    qdd = forward_dynamics(model, x, u, gravity)
    return x + dt * np.concatenate([x[:, n:], qdd], axis=1)


def euler_gradient(model, x, u, dt, gravity=-9.81):
    """TrajoptPlant.integrator type 0, return_gradient=True (:100-108) -> A (K,nx,nx), B (K,nx,nu)."""
    n = model.n
    K = x.shape[0]
    dqdd = forward_dynamics_gradient(model, x, u, gravity)
    top = np.concatenate([np.zeros((n, n)), np.eye(n), np.zeros((n, n))], axis=1)
    dxdot = np.concatenate([np.broadcast_to(top, (K, n, 3 * n)), dqdd], axis=1)
    A = np.eye(2 * n)[None] + dt * dxdot[:, :, :2 * n]
    B = dt * dxdot[:, :, 2 * n:]
    return A, B
