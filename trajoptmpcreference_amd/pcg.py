"""PCG -- the GBD-PCG-Python solver class (GBD-PCG-Python/PCG.py:4-215) on
the GPU.

Same constructor and ``solve()`` contract: ``PCG(A, b, block_size, Nblocks,
guess=None, options={}).solve()`` returns ``(x, (trace_nu, trace_res))`` with
x a column vector, trace_nu = |rho_k| per iteration (PCG.py:82,94,110) and
trace_res = ||b - A x_k|| (:83,95).  A must be block-tridiagonal with blocks of
``block_size`` (the Schur complement of the trajectory KKT system); the blocks
are extracted at this boundary and the solve runs in libtmpc's one-workgroup-
per-system kernel.  Invalid options raise ValueError instead of exit().
"""
import numpy as np

from . import _native

VALID_PRECONDITIONERS = ("0", "J", "BJ", "SS")


def extract_blocks(A, block_size):
    """Diagonal, sub- and super-diagonal blocks of a block-tridiagonal matrix."""
    A = np.asarray(A, dtype=np.float64)
    n = A.shape[0]
    if A.shape != (n, n) or n % block_size:
        raise ValueError(f"A must be square with a dimension divisible by block_size={block_size}, got {A.shape}")
    N = n // block_size
    b = block_size
    Dg = np.array([A[k * b:(k + 1) * b, k * b:(k + 1) * b] for k in range(N)])
    Lo = np.array([A[(k + 1) * b:(k + 2) * b, k * b:(k + 1) * b] for k in range(N - 1)]).reshape(max(N - 1, 0), b, b)
    Up = np.array([A[k * b:(k + 1) * b, (k + 1) * b:(k + 2) * b] for k in range(N - 1)]).reshape(max(N - 1, 0), b, b)
    mask = np.zeros((N, N), dtype=bool)
    for k in range(N):
        mask[k, max(0, k - 1):min(N, k + 2)] = True
    outside = np.kron(~mask, np.ones((b, b), dtype=bool))
    if np.any(A[outside] != 0):
        raise ValueError("A is not block-tridiagonal with the given block_size")
    return Dg, Lo, Up


class PCG:
    def __init__(self, A, b, block_size, Nblocks, guess=None, options=None, overloading=False, device=0):
        self.A = A
        self.b = b
        self.block_size = int(block_size)
        self.Nblocks = Nblocks
        self.guess = guess
        self.options = {} if options is None else options
        self.overloading = overloading
        self.device = device
        self.set_default_options(self.options)
        self._Pd = None

    def set_default_options(self, options):
        """PCG.py:19-25."""
        options.setdefault("exit_tolerance", 1e-6)
        options.setdefault("max_iter", 100)
        options.setdefault("DEBUG_MODE", False)
        options.setdefault("RETURN_TRACE", False)
        options.setdefault("preconditioner_type", "BJ")
        self.validate_precon_type(options["preconditioner_type"])

    def validate_precon_type(self, precon_type):
        if precon_type not in VALID_PRECONDITIONERS:
            raise ValueError("Invalid preconditioner options are [0: none, J : Jacobi, BJ: Block-Jacobi, "
                             "SS: Symmetric Stair]")

    def update_A(self, A):
        self.A = A

    def update_b(self, b):
        self.b = b

    def update_guess(self, guess):
        self.guess = guess

    def update_exit_tolerance(self, tol):
        self.options["exit_tolerance"] = tol

    def update_max_iter(self, max_iter):
        self.options["max_iter"] = max_iter

    def update_preconditioner_type(self, type):
        self.validate_precon_type(type)
        self.options["preconditioner_type"] = type

    def update_DEBUG_MODE(self, mode):
        self.options["DEBUG_MODE"] = mode

    def update_RETURN_TRACE(self, mode):
        self.options["RETURN_TRACE"] = mode

    def solve(self):
        Dg, Lo, Up = extract_blocks(self.A, self.block_size)
        N, nx = Dg.shape[0], self.block_size
        b = np.asarray(self.b, dtype=np.float64).reshape(1, -1)
        guess = None
        if self.guess is not None:
            g = np.asarray(self.guess, dtype=np.float64).reshape(1, -1)
            if np.any(g != 0):
                guess = g
        max_iter = int(self.options["max_iter"])
        ctx = _native.default_context(self.device)
        lam, it, tn, tr, Pd = ctx.pcg_batch(Dg[None], Lo[None], b, precond=self.options["preconditioner_type"],
                                            S_up=Up[None], guess=guess, tol=float(self.options["exit_tolerance"]),
                                            max_iter=max_iter, trace=True)
        self._Pd = Pd[0]
        n_it = int(it[0])
        self.iterations = n_it
        trace = [float(v) for v in tn[0, :n_it + 1]]
        trace2 = [float(v) for v in tr[0, :n_it + 1]]
        return lam[0].reshape(-1, 1), (trace, trace2)

    @property
    def Pinv(self):
        """Dense preconditioner as compute_preconditioner builds it (PCG.py:166-212)."""
        Dg, Lo, Up = extract_blocks(self.A, self.block_size)
        N, b = Dg.shape[0], self.block_size
        ptype = self.options["preconditioner_type"]
        P = np.zeros((N * b, N * b))
        if ptype == "J":
            return np.diag(1.0 / np.diag(np.asarray(self.A, dtype=np.float64)))
        if ptype == "0":   # identity (PCG.py:114-118)
            return np.identity(N * b)
        if self._Pd is None:
            self.solve()
        Pd = self._Pd
        for k in range(N):
            P[k * b:(k + 1) * b, k * b:(k + 1) * b] = Pd[k]
        if ptype == "SS":
            for k in range(N):
                if k % 2:
                    lo = -Pd[k] @ (Lo[k - 1] @ Pd[k - 1])
                    P[k * b:(k + 1) * b, (k - 1) * b:k * b] = lo
                    P[(k - 1) * b:k * b, k * b:(k + 1) * b] = lo.T
                    if k < N - 1:
                        up = -Pd[k] @ (Up[k] @ Pd[k + 1])
                        P[k * b:(k + 1) * b, (k + 1) * b:(k + 2) * b] = up
                        P[(k + 1) * b:(k + 2) * b, k * b:(k + 1) * b] = up.T
        return P
