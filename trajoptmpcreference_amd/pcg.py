"""PCG -- the GBD-PCG-Python solver class (GBD-PCG-Python/PCG.py:4-215) on
the GPU.

Same constructor and ``solve()`` contract: ``PCG(A, b, block_size, Nblocks,
guess=None, options={}).solve()`` returns ``(x, (trace_nu, trace_res))`` with
x a column vector, trace_nu = |rho_k| per iteration (PCG.py:82,94,110) and
trace_res = ||b - A x_k|| (:83,95).  A block-tridiagonal A of at most 1024 rows
(the Schur complement of the trajectory KKT system) runs in libtmpc's fused
one-workgroup-per-system kernel on its blocks; any other A, and
``pcg(A, b, Pinv, guess, options)`` with any preconditioner matrix, run the
dense device PCG (tmpc_pcg_dense_batch, any size).  Invalid options
raise ValueError instead of exit().
"""
import numpy as np

from . import _native
from ._options import NO_OPTIONS, fresh

VALID_PRECONDITIONERS = ("0", "J", "BJ", "SS")
FUSED_MAX_ROWS = 1024   # tmpc_pcg_batch: one row of S per lane of one workgroup
DENSE_MAX_ROWS = 4096   # tmpc_pcg_dense_batch's one-workgroup kernel; past it the multi-launch form


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
    def __init__(self, A, b, block_size, Nblocks, guess=None, options=NO_OPTIONS, overloading=False, device=0):
        self.A = A
        self.b = b
        self.block_size = int(block_size)
        self.Nblocks = Nblocks
        self.guess = guess
        self.options = fresh(options)
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

    def _run(self, A, b, guess, options):
        """PCG.solve: the fused block-tridiagonal kernel (tmpc_pcg_batch) where A is block-tridiagonal with
        at most 1024 rows, else the dense PCG with the block preconditioner built on the device
        (tmpc_pcg_dense_batch, any size)."""
        A = np.asarray(A, dtype=np.float64)
        n = A.shape[0]
        if n > FUSED_MAX_ROWS or A.shape != (n, n) or n % self.block_size:
            return self._run_dense(A, b, None, guess, options)
        try:
            Dg, Lo, Up = extract_blocks(A, self.block_size)
        except ValueError:
            return self._run_dense(A, b, None, guess, options)
        b = np.asarray(b, dtype=np.float64).reshape(1, -1)
        if guess is not None:
            g = np.asarray(guess, dtype=np.float64).reshape(1, -1)
            guess = g if np.any(g != 0) else None
        max_iter = int(options["max_iter"])
        ctx = _native.default_context(self.device)
        lam, it, tn, tr, Pd = ctx.pcg_batch(Dg[None], Lo[None], b, precond=options["preconditioner_type"],
                                            S_up=Up[None], guess=guess, tol=float(options["exit_tolerance"]),
                                            max_iter=max_iter, trace=True)
        n_it = int(it[0])
        self.iterations = n_it
        trace = [float(v) for v in tn[0, :n_it + 1]]
        trace2 = [float(v) for v in tr[0, :n_it + 1]]
        return lam[0].reshape(-1, 1), (trace, trace2), Pd[0]

    def _run_dense(self, A, b, Pinv, guess, options):
        """PCG.pcg on the dense A with the preconditioner matrix Pinv (None: options['preconditioner_type']
        with this object's block size, built on the device) -- tmpc_pcg_dense_batch."""
        A = np.asarray(A, dtype=np.float64)
        n = A.shape[0]
        if A.shape != (n, n):
            raise ValueError(f"A must be square, got {A.shape}")
        b = np.asarray(b, dtype=np.float64).reshape(1, -1)
        g = None
        if guess is not None:
            g = np.asarray(guess, dtype=np.float64).reshape(1, -1)
            g = g if np.any(g != 0) else None
        if Pinv is not None:
            Pinv = np.asarray(Pinv, dtype=np.float64)
            if Pinv.shape != (n, n):
                raise ValueError(f"Pinv must be {(n, n)}, got {Pinv.shape}")
            Pinv = Pinv[None]
        max_iter = int(options["max_iter"])
        ctx = _native.default_context(self.device)
        x, it, tn, tr, _ = ctx.pcg_dense_batch(A[None], b, Pinv, precond=options["preconditioner_type"],
                                               nx=self.block_size, guess=g, tol=float(options["exit_tolerance"]),
                                               max_iter=max_iter)
        n_it = int(it[0])
        self.iterations = n_it
        trace = [float(v) for v in tn[0, :n_it + 1]]
        trace2 = [float(v) for v in tr[0, :n_it + 1]]
        return x[0].reshape(-1, 1), (trace, trace2), None

    def solve(self):
        """PCG.solve (PCG.py:214-215): pcg(A, b, Pinv, guess, options) with this object's preconditioner."""
        x, traces, self._Pd = self._run(self.A, self.b, self.guess, self.options)
        return x, traces

    def pcg(self, A, b, Pinv, guess, options=NO_OPTIONS):
        """PCG.pcg (PCG.py:66-111) with the caller's preconditioner matrix, whatever it is: z = Pinv r on
        the device (tmpc_pcg_dense_batch, any size)."""
        options = fresh(options)
        self.set_default_options(options)
        x, traces, _ = self._run_dense(A, b, Pinv, guess, options)
        return x, traces

    def compute_preconditioner(self, A, block_size, preconditioner_type):
        """PCG.compute_preconditioner (PCG.py:113-212) as a dense matrix: '0' identity, J diag(A)^-1, BJ the
        inverses of the floor(n / block_size) diagonal blocks, SS the symmetric stair (odd block rows carry
        -P_k A_k,k+-1 P_k+-1, mirrored to the even ones) -- built on the device from A (the dense PCG's
        builder, k_dense_gj / k_dense_stair), any A."""
        self.validate_precon_type(preconditioner_type)
        A = np.asarray(A, dtype=np.float64)
        n = A.shape[0]
        if preconditioner_type == "0":
            return np.identity(n)
        if A.shape != (n, n):
            raise ValueError(f"A must be square, got {A.shape}")
        ctx = _native.default_context(self.device)
        _, _, _, _, P = ctx.pcg_dense_batch(A[None], np.zeros((1, n)), None, precond=preconditioner_type,
                                            nx=int(block_size), tol=1.0, max_iter=0, trace=False, want_pinv=True)
        return P[0]

    @property
    def Pinv(self):
        """The dense preconditioner (the reference's self.Pinv, PCG.py:16)."""
        return self.compute_preconditioner(self.A, self.block_size, self.options["preconditioner_type"])
