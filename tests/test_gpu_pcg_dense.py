"""GPU parity: the dense PCG (tmpc_pcg_dense_batch) -- PCG.pcg(A, b, Pinv, guess, options)
(GBD-PCG-Python/PCG.py:66-111) with ANY preconditioner matrix, and PCG.solve past the fused kernel's 1024
rows with the block preconditioner built on the device (compute_preconditioner, PCG.py:113-212).

* On the reference's own Schur complements and preconditioner matrices (tests/golden/qp_*.npz): the
  iteration count is the reference's exactly, for 0 / J / BJ / SS and from the reference's warm start;
  x and the |nu| trace bit for bit against oracle/dense.py (the kernel's operation order, itself pinned
  to the reference on the CPU: test_oracle_dense.py), ||b - A x|| within 1e-14 relative (a square root
  of the same sum).
* The preconditioner the device builds equals oracle/dense.py block_pinv bit for bit, and the
  reference's to 1e-12.
* Arbitrary Pinv (no block structure) and dimensions past 1024 rows, including a trailing partial block,
  through the PCG class: bit for bit against the oracle.
* Past 4096 rows (the multi-launch form, vectors in HBM; round 6): the same operation order, bit for bit
  against the oracle through the PCG class, with an arbitrary Pinv in a batch of two, and from a guess."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

FIX = ["qp_arm2_N8", "qp_arm3_N32", "qp_arm6fix_N64"]


def _system(d):
    from oracle import dense as od
    return od.from_blocks(d["S_diag"], d["S_lo"], d["S_up"]), np.asarray(d["gamma"], dtype=float).reshape(-1)


def _ref_pinv(d, ptype):
    from oracle import dense as od
    if ptype == "0":
        return np.identity(d["S_diag"].shape[0] * d["S_diag"].shape[1])
    return od.from_blocks(d[f"P_{ptype}_diag"], d[f"P_{ptype}_lo"], d[f"P_{ptype}_up"])


def _same(gpu, ora, it):
    x, n, tn, tr = gpu
    xo, no, tno, tro = ora
    assert int(n) == no
    assert np.array_equal(x, xo)
    assert np.array_equal(tn[:no + 1], np.array(tno))
    assert np.allclose(tr[:no + 1], np.array(tro), rtol=1e-14, atol=0)


@pytest.mark.parametrize("name", FIX)
@pytest.mark.parametrize("ptype", ["J", "BJ", "SS", "0"])
def test_dense_pcg_with_the_references_pinv(name, ptype):
    from oracle import dense as od
    from trajoptmpcreference_amd import _native
    d = golden(f"{name}.npz")
    S, g = _system(d)
    P = _ref_pinv(d, ptype)
    ctx = _native.default_context(0)
    x, it, tn, tr, _ = ctx.pcg_dense_batch(S[None], g[None], P[None])
    assert int(it[0]) == int(d[f"iters_{ptype}"])
    _same((x[0], it[0], tn[0], tr[0]), od.pcg(S, g, P), None)


@pytest.mark.parametrize("name", FIX)
@pytest.mark.parametrize("ptype", ["J", "BJ", "SS", "0"])
def test_dense_pcg_with_the_device_block_preconditioner(name, ptype):
    from oracle import dense as od
    from trajoptmpcreference_amd import _native
    d = golden(f"{name}.npz")
    S, g = _system(d)
    nx = d["S_diag"].shape[1]
    ctx = _native.default_context(0)
    x, it, tn, tr, P = ctx.pcg_dense_batch(S[None], g[None], None, precond=ptype, nx=nx, want_pinv=True)
    Po = od.block_pinv(S, nx, ptype)
    assert np.array_equal(P[0], Po)
    if ptype in ("BJ", "SS"):
        assert float(np.max(np.abs(P[0] - _ref_pinv(d, ptype)))) <= 1e-12 * float(np.max(np.abs(Po)))
    assert int(it[0]) == int(d[f"iters_{ptype}"])
    _same((x[0], it[0], tn[0], tr[0]), od.pcg(S, g, Po), None)


@pytest.mark.parametrize("name", FIX)
@pytest.mark.parametrize("ptype", ["BJ", "SS"])
def test_dense_pcg_warm_start(name, ptype):
    from oracle import dense as od
    from trajoptmpcreference_amd import _native
    d = golden(f"{name}.npz")
    S, g = _system(d)
    P = _ref_pinv(d, ptype)
    ctx = _native.default_context(0)
    x, it, tn, tr, _ = ctx.pcg_dense_batch(S[None], g[None], P[None], guess=np.asarray(d["guess"]).reshape(1, -1))
    assert int(it[0]) == int(d[f"iters_{ptype}_guess"])
    _same((x[0], it[0], tn[0], tr[0]), od.pcg(S, g, P, guess=d["guess"]), None)


def _random_system(D, nx, seed, width=None):
    """a negative definite block-tridiagonal (width None) or banded system with its right-hand side"""
    rng = np.random.default_rng(seed)
    if width is None:
        M = np.zeros((D, D))
        for k in range(D // nx + 1):
            r0, r1 = k * nx, min(D, (k + 1) * nx)
            c0 = max(0, r0 - nx)
            M[r0:r1, c0:r1] = rng.uniform(-1.0, 1.0, (r1 - r0, r1 - c0))
    else:
        M = np.zeros((D, D))
        for o in range(-width, width + 1):
            M += np.diag(rng.uniform(-1.0, 1.0, D - abs(o)), o)
    S = -(M @ M.T + 2.0 * np.eye(D))
    return S, rng.uniform(-1.0, 1.0, D)


def test_arbitrary_pinv_and_batches():
    """A preconditioner matrix with no block structure (a symmetric perturbation of the inverse of S's
    diagonal, dense), two systems of one batch with different preconditioners: bit for bit per system."""
    from oracle import dense as od
    from trajoptmpcreference_amd import _native
    D = 200
    S0, g0 = _random_system(D, 10, 3)
    S1, g1 = _random_system(D, 10, 4, width=7)
    rng = np.random.default_rng(5)
    E = rng.uniform(-1.0, 1.0, (D, D)) * 1e-3
    P0 = np.diag(1.0 / np.diag(S0)) + (E + E.T)
    P1 = od.block_pinv(S1, 10, "SS")
    ctx = _native.default_context(0)
    x, it, tn, tr, _ = ctx.pcg_dense_batch(np.stack([S0, S1]), np.stack([g0, g1]), np.stack([P0, P1]), tol=1e-10,
                                           max_iter=300)
    for i, (S, g, P) in enumerate(((S0, g0, P0), (S1, g1, P1))):
        ora = od.pcg(S, g, P, tol=1e-10, max_iter=300)
        assert 3 < ora[1] < 300
        _same((x[i], it[i], tn[i], tr[i]), ora, None)


@pytest.mark.parametrize("D,nx,ptype", [(1792, 14, "SS"), (1530, 12, "BJ"), (2100, 14, "SS")])
def test_pcg_class_past_the_fused_rows(D, nx, ptype):
    """PCG(A, b, nx, N, options).solve() past 1024 rows (a 7-joint arm's Schur dimension at N = 128; a
    trailing partial block at 1530 = 127 x 12 + 6) and .pcg with the class's own Pinv: the dense device
    path, bit for bit against the oracle with the canonical block preconditioner."""
    from oracle import dense as od
    from trajoptmpcreference_amd import PCG
    S, g = _random_system(D, nx, D)
    opts = {"preconditioner_type": ptype, "exit_tolerance": 1e-8, "max_iter": 200}
    pcg = PCG(S, g.reshape(-1, 1), nx, D // nx, options=dict(opts))
    x, (trace, trace2) = pcg.solve()
    Po = od.block_pinv(S, nx, ptype)
    xo, no, tno, tro = od.pcg(S, g, Po, tol=1e-8, max_iter=200)
    assert 5 < no < 200
    assert len(trace) == no + 1 and np.array_equal(x.reshape(-1), xo)
    assert np.array_equal(np.array(trace), np.array(tno))
    P = pcg.compute_preconditioner(S, nx, ptype)
    assert np.array_equal(P, Po)
    x2, (trace2b, _) = pcg.pcg(S, g.reshape(-1, 1), P, np.zeros(D), dict(opts))
    assert np.array_equal(x2.reshape(-1), xo) and len(trace2b) == no + 1


def test_pcg_class_past_4096_rows():
    """PCG(A, b, nx, N).solve() at 5000 rows (10-row blocks, SS) and compute_preconditioner: the
    multi-launch device PCG, iteration count, x and the |nu| trace bit for bit against the oracle."""
    from oracle import dense as od
    from trajoptmpcreference_amd import PCG
    D, nx = 5000, 10
    S, g = _random_system(D, nx, 17)
    opts = {"preconditioner_type": "SS", "exit_tolerance": 1e-8, "max_iter": 150}
    pcg = PCG(S, g.reshape(-1, 1), nx, D // nx, options=dict(opts))
    x, (trace, trace2) = pcg.solve()
    Po = od.block_pinv(S, nx, "SS")
    xo, no, tno, tro = od.pcg(S, g, Po, tol=1e-8, max_iter=150)
    assert 5 < no < 150
    assert len(trace) == no + 1 and np.array_equal(x.reshape(-1), xo)
    assert np.array_equal(np.array(trace), np.array(tno))
    assert np.allclose(np.array(trace2), np.array(tro), rtol=1e-14, atol=0)
    assert np.array_equal(pcg.compute_preconditioner(S, nx, "SS"), Po)


def test_dense_pcg_past_4096_rows_arbitrary_pinv_batch_and_guess():
    """Two 4200-row systems in one batch -- a dense arbitrary Pinv and the device's BJ blocks of a banded
    system -- from a nonzero guess: per system bit for bit against the oracle; the system that converges
    first stops (its later launches return) while the other continues."""
    from oracle import dense as od
    from trajoptmpcreference_amd import _native
    D = 4200
    S0, g0 = _random_system(D, 12, 31)
    S1, g1 = _random_system(D, 12, 32, width=9)
    rng = np.random.default_rng(33)
    E = rng.uniform(-1.0, 1.0, (D, D)) * 1e-4
    P0 = np.diag(1.0 / np.diag(S0)) + (E + E.T)
    P1 = od.block_pinv(S1, 12, "BJ")
    guess = rng.uniform(-0.1, 0.1, (2, D))
    ctx = _native.default_context(0)
    x, it, tn, tr, _ = ctx.pcg_dense_batch(np.stack([S0, S1]), np.stack([g0, g1]), np.stack([P0, P1]), guess=guess,
                                           tol=1e-9, max_iter=400)
    counts = []
    for i, (S, g, P) in enumerate(((S0, g0, P0), (S1, g1, P1))):
        ora = od.pcg(S, g, P, guess=guess[i], tol=1e-9, max_iter=400)
        assert 3 < ora[1] < 400
        _same((x[i], it[i], tn[i], tr[i]), ora, None)
        counts.append(ora[1])
    assert counts[0] != counts[1]
