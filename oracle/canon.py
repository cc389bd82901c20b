"""ORACLE -- test infrastructure (see oracle/__init__.py): ctypes binding of oracle/libcanon.so
(oracle/canon.c, built by `make -C oracle` / __graft_entry__.build()), the PCG of
GBD-PCG-Python/PCG.py:66-212 in the canonical operation order of the GPU's fused QP kernel, in
both of its lane layouts (one row of S per lane; two rows per lane -- the register instance past
768 rows and the HBM-row "GM" instance)."""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
PRECOND = {"J": 1, "BJ": 2, "SS": 3, "0": 4}
# the kernel's layout thresholds (csrc/tmpc_kernels.hip pcg_rpl, LaunchNJ::qp; csrc/tmpc_internal.h)
RPL1_MAX_ROWS = 768
REG_MAX_ROWS = 1024


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libcanon.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path}: build it with `make -C oracle` (or __graft_entry__.build())")
        lib = C.CDLL(path)
        dp = C.POINTER(C.c_double)
        lib.canon_pcg.restype = C.c_int
        lib.canon_pcg.argtypes = [C.c_int, C.c_int, C.c_int, dp, dp, dp, C.c_double, C.c_int, dp, dp]
        lib.canon_pcg_rpl.restype = C.c_int
        lib.canon_pcg_rpl.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, dp, dp, dp, dp, C.c_double, C.c_int,
                                      dp, dp]
        lib.canon_block_inverse.restype = C.c_int
        lib.canon_block_inverse.argtypes = [C.c_int, C.c_int, dp, dp]
        _LIB = lib
    return _LIB


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double)) if a is not None else None


def qp_rpl(N, nx, gm_min_rows=None):
    """Rows of S per lane of the fused QP kernel's PCG for an N-block system (LaunchNJ::qp): the GM
    instance (past 1024 rows, or from `gm_min_rows` rows when TMPC_QP_GM_MIN_ROWS forces it) and the
    register instance past 768 rows take two; otherwise one."""
    rows = N * nx
    gm = rows > REG_MAX_ROWS or (gm_min_rows is not None and rows >= gm_min_rows)
    if gm:
        return 2
    return 1 if (rows <= RPL1_MAX_ROWS or nx % 2) else 2


def pcg(S_diag, S_lo, gamma, ptype, tol=1e-6, max_iter=100, rpl=None, guess=None):
    """S_diag [N][nx][nx], S_lo [N-1][nx][nx] (S_{k+1,k}), gamma [N nx] -> (lambda, iterations, |nu| trace).
    rpl: the kernel's rows per lane (default: the fused QP kernel's register layout for this size,
    qp_rpl); guess: the warm-start iterate (PCG.py:11-12)."""
    Sd = np.ascontiguousarray(S_diag, dtype=np.float64)
    N, nx, _ = Sd.shape
    Sl = np.ascontiguousarray(S_lo if N > 1 else np.zeros((1, nx, nx)), dtype=np.float64)
    b = np.ascontiguousarray(gamma, dtype=np.float64).reshape(-1)
    if rpl is None:
        rpl = qp_rpl(N, nx)
    g = None if guess is None else np.ascontiguousarray(guess, dtype=np.float64).reshape(-1)
    x = np.zeros(N * nx)
    tn = np.full(max_iter + 1, np.nan)
    it = _lib().canon_pcg_rpl(N, nx, PRECOND[ptype], int(rpl), _p(Sd), _p(Sl), _p(b), _p(g), float(tol),
                              int(max_iter), _p(x), _p(tn))
    if it < 0:
        raise ValueError(f"canon_pcg_rpl: unsupported size N={N} nx={nx} rpl={rpl} (<= 1024 lanes) "
                         f"or allocation failure ({it})")
    return x, it, tn[:it + 1]


def block_inverse(S_diag):
    """(S_kk)^-1 per block by the kernel's Gauss-Jordan (the BJ / SS preconditioner blocks)."""
    Sd = np.ascontiguousarray(S_diag, dtype=np.float64)
    N, nx, _ = Sd.shape
    P = np.zeros_like(Sd)
    _lib().canon_block_inverse(N, nx, _p(Sd), _p(P))
    return P
