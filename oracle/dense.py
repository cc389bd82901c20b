"""TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product): a restatement of the dense PCG
of tmpc_pcg_dense_batch (csrc/tmpc_hard.hip: k_pcg_dense, k_dense_gj, k_dense_stair) in its own
operation order, so the GPU can be checked bit for bit on identical inputs.

GBD-PCG-Python/PCG.py:66-111 (PCG.pcg(A, b, Pinv, guess, options)): any dense A and preconditioner
matrix Pinv, any dimension.  The canonical order of the device kernel:
  * every matrix-vector product y = M v sequential over the columns from 0.0, each product and sum
    rounded on its own (y = y + M[:, c] * v[c], c = 0, 1, ...);
  * every dot product as oracle/hard.py _dot (1024 per-thread partials, the 64-lane xor butterfly, the
    16-wave fan-in) -- the hard-limit PCG's workgroup;
  * r0 = b - A x0, trace_res = sqrt(r . r) of the explicit b - A x_k (PCG.py:83, 95), trace_nu = |nu|;
  * the block preconditioner of PCG.solve (compute_preconditioner, PCG.py:113-212), when the caller
    gives none, from oracle/hard.py preconditioner_canonical, placed in a dense matrix.
Parity with the reference's own NumPy order is anchored by the PCG fixtures (tests/golden/pcg_*.npz):
counts identical there (tests/test_oracle_dense.py)."""
import numpy as np

from .hard import _dot, preconditioner_canonical


def matvec(M, v):
    """M v, sequential over the columns from 0.0 (the device's order)"""
    M = np.asarray(M, dtype=float)
    s = np.zeros(M.shape[0])
    for c in range(M.shape[1]):
        s = s + M[:, c] * v[c]
    return s


def from_blocks(Dg, Lo, Up=None):
    """the dense block-tridiagonal matrix of diagonal blocks Dg [N][b][b], sub-diagonal Lo [N-1][b][b]
    (block (k+1, k)) and super-diagonal Up (block (k, k+1); None: Lo^T)"""
    Dg = np.asarray(Dg, dtype=float)
    N, b = Dg.shape[0], Dg.shape[1]
    M = np.zeros((N * b, N * b))
    for k in range(N):
        M[k * b:(k + 1) * b, k * b:(k + 1) * b] = Dg[k]
    for k in range(N - 1):
        M[(k + 1) * b:(k + 2) * b, k * b:(k + 1) * b] = Lo[k]
        M[k * b:(k + 1) * b, (k + 1) * b:(k + 2) * b] = Lo[k].T if Up is None else Up[k]
    return M


def block_pinv(A, nx, ptype):
    """compute_preconditioner (PCG.py:113-212) as a dense matrix from preconditioner_canonical's blocks:
    '0' identity, 'J' 1 / diag(A), 'BJ' / 'SS' the nx-aligned blocks from row 0 (rows past the last full
    block: zero, PCG.py:182)."""
    A = np.asarray(A, dtype=float)
    D = A.shape[0]
    if ptype == "0":
        return np.identity(D)
    if ptype == "J":
        P = np.zeros((D, D))
        for a in range(D):
            P[a, a] = 1.0 / A[a, a]
        return P
    Pd, Pl = preconditioner_canonical(A, nx, ptype)
    nb = D // nx
    P = np.zeros((D, D))
    for k in range(nb):
        P[k * nx:(k + 1) * nx, k * nx:(k + 1) * nx] = Pd[k]
    if ptype == "SS":
        for k in range(nb - 1):   # Pl[k] = P_{k+1,k}; P_{k,k+1} = Pl[k]^T
            P[(k + 1) * nx:(k + 2) * nx, k * nx:(k + 1) * nx] = Pl[k]
            P[k * nx:(k + 1) * nx, (k + 1) * nx:(k + 2) * nx] = Pl[k].T
    return P


def pcg(A, b, Pinv, guess=None, tol=1e-6, max_iter=100):
    """PCG.pcg in the device's order.  Returns (x, iterations, trace_nu, trace_res)."""
    A = np.asarray(A, dtype=float)
    Pinv = np.asarray(Pinv, dtype=float)
    b = np.asarray(b, dtype=float).reshape(-1)
    x = np.zeros_like(b) if guess is None else np.array(guess, dtype=float).reshape(-1)
    r = b - matvec(A, x)
    trace_res = [float(np.sqrt(_dot(r, r)))]
    z = matvec(Pinv, r)
    p = z.copy()
    nu = _dot(r, z)
    trace_nu = [abs(nu)]
    it_done = max_iter
    for it in range(max_iter):
        Ap = matvec(A, p)
        alpha = nu / _dot(p, Ap)
        r = r - Ap * alpha
        x = x + p * alpha
        z = matvec(Pinv, r)
        nup = _dot(r, z)
        res = b - matvec(A, x)
        trace_nu.append(abs(nup))
        trace_res.append(float(np.sqrt(_dot(res, res))))
        if abs(nup) < tol:
            it_done = it + 1
            break
        beta = nup / nu
        p = z + p * beta
        nu = nup
    return x, it_done, trace_nu, trace_res
