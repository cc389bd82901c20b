"""GPU parity: block-tridiagonal PCG (tmpc_pcg_batch, the PCG class) and one
full QP (tmpc_qp_batch: dynamics + Schur + PCG + dxu) against the reference.

Fixtures qp_*.npz hold the reference's dense S, P^-1 (as blocks), gamma,
lambda, PCG traces and dxul at the first QP of the §8d workload.
Iteration counts must be identical (integer parity); floating point within
the stated tolerances (relative to the magnitude of each quantity).
"""
import numpy as np
import pytest

from conftest import arm_model, golden, quad_cost_arrays

pytestmark = pytest.mark.gpu

CASES = [("arm2", 8), ("arm3", 32), ("arm6fix", 64)]


def _rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b)))) / max(1.0, float(np.max(np.abs(b))))


@pytest.mark.parametrize("name,N", CASES)
@pytest.mark.parametrize("pre", ["J", "BJ", "SS", "0"])
def test_pcg_on_reference_blocks(ctx, name, N, pre):
    d = golden(f"qp_{name}_N{N}.npz")
    lam, it, tn, tr, Pd = ctx.pcg_batch(d["S_diag"][None], d["S_lo"][None], d["gamma"][None], precond=pre,
                                        S_up=d["S_up"][None], tol=1e-6, max_iter=100)
    assert int(it[0]) == int(d[f"iters_{pre}"])
    n_it = int(it[0])
    # |nu| trace: relative agreement early, absolute near the 1e-6 exit threshold
    ref_tn = d[f"trace_nu_{pre}"]
    nt = 10 if pre == "0" else n_it + 1   # '0': late trace rounding-sensitive (test_oracle_golden)
    assert np.allclose(tn[0, :nt], ref_tn[:nt], rtol=1e-6, atol=1e-9)
    assert _rel(lam[0], d[f"lam_{pre}"]) < (1e-6 if pre in ("J", "0") else 1e-8)
    if pre != "J":
        assert _rel(Pd[0], d[f"P_{pre}_diag"]) < 1e-10


@pytest.mark.parametrize("name,N", CASES)
@pytest.mark.parametrize("pre", ["J", "BJ", "SS", "0"])
def test_pcg_bitwise_canonical(ctx, name, N, pre):
    """The kernel is the canonical-order restatement (oracle/canon.c) bit for bit on identical inputs:
    iteration count, lambda, the |nu| trace and the preconditioner blocks (S_{k,k+1} = S_{k+1,k}^T, as the
    fused QP kernel forms it)."""
    from oracle import canon
    d = golden(f"qp_{name}_N{N}.npz")
    lam, it, tn, _, Pd = ctx.pcg_batch(d["S_diag"][None], d["S_lo"][None], d["gamma"][None], precond=pre,
                                       tol=1e-6, max_iter=100)
    lam_c, it_c, tn_c = canon.pcg(d["S_diag"], d["S_lo"], d["gamma"], pre)
    assert int(it[0]) == it_c == int(d[f"iters_{pre}"])
    assert np.array_equal(lam[0], lam_c)
    assert np.array_equal(tn[0, :it_c + 1], tn_c)
    if pre in ("BJ", "SS"):
        assert np.array_equal(Pd[0], canon.block_inverse(d["S_diag"]))


@pytest.mark.parametrize("name,N", CASES)
@pytest.mark.parametrize("pre", ["BJ", "SS"])
def test_pcg_guess_matches_reference(ctx, name, N, pre):
    """PCG.update_guess (TrajoptMPCReference.py:439-440): the reference's solve from a given x0."""
    d = golden(f"qp_{name}_N{N}.npz")
    lam, it, tn, _, _ = ctx.pcg_batch(d["S_diag"][None], d["S_lo"][None], d["gamma"][None], precond=pre,
                                      S_up=d["S_up"][None], guess=d["guess"][None], tol=1e-6, max_iter=100)
    assert int(it[0]) == int(d[f"iters_{pre}_guess"])
    n_it = int(it[0])
    assert np.allclose(tn[0, :n_it + 1], d[f"trace_nu_{pre}_guess"], rtol=1e-6, atol=1e-9)
    assert _rel(lam[0], d[f"lam_{pre}_guess"]) < 1e-8


@pytest.mark.parametrize("name,N", CASES)
def test_qp_guess_matches_reference(ctx, name, N):
    """solveKKTSystem_Schur(options={'guess': g}) -> the fused QP kernel starts its PCG at g."""
    d = golden(f"qp_{name}_N{N}.npz")
    m = arm_model(name)
    ctx.set_model(m)
    ctx.set_cost_quadratic(*quad_cost_arrays(m.n))
    r = ctx.qp_batch(d["x"][None], d["u"][None], N, float(d["dt"]), float(d["rho"]), "PCG-SS", want_blocks=False,
                     guess=d["guess"][None])
    assert int(r["pcg_iters"][0]) == int(d["iters_SS_guess"])
    assert _rel(r["dxul"][0], d["dxul_SS_guess"]) < 1e-7


@pytest.mark.parametrize("name,N", CASES)
def test_pcg_class_api(name, N):
    from trajoptmpcreference_amd import PCG
    from oracle.sqp import dense_from_blocks
    d = golden(f"qp_{name}_N{N}.npz")
    S = dense_from_blocks(d["S_diag"], d["S_lo"], d["S_up"])
    nx = d["S_diag"].shape[1]
    pcg = PCG(S, d["gamma"].reshape(-1, 1), nx, N, options={"preconditioner_type": "SS"})
    lam, (trace, trace2) = pcg.solve()
    assert lam.shape == (N * nx, 1)
    assert len(trace) - 1 == int(d["iters_SS"])
    assert np.allclose(trace2, d["trace_res_SS"], rtol=1e-5, atol=1e-9)
    P = pcg.Pinv
    Pref = dense_from_blocks(d["P_SS_diag"], d["P_SS_lo"], d["P_SS_up"])
    assert _rel(P, Pref) < 1e-10


@pytest.mark.parametrize("name,N", CASES)
@pytest.mark.parametrize("pre", ["J", "BJ", "SS"])
def test_qp_matches_reference(ctx, name, N, pre):
    d = golden(f"qp_{name}_N{N}.npz")
    m = arm_model(name)
    ctx.set_model(m)
    ctx.set_cost_quadratic(*quad_cost_arrays(m.n))
    r = ctx.qp_batch(d["x"][None], d["u"][None], N, float(d["dt"]), float(d["rho"]), "PCG-" + pre)
    assert _rel(r["S_diag"][0], d["S_diag"]) < 1e-11
    assert _rel(r["S_lo"][0], d["S_lo"]) < 1e-11
    assert _rel(r["gamma"][0], d["gamma"]) < 1e-11
    assert int(r["pcg_iters"][0]) == int(d[f"iters_{pre}"])
    assert _rel(r["dxul"][0], d[f"dxul_{pre}"]) < (1e-5 if pre == "J" else 1e-7)


@pytest.mark.parametrize("name,N", CASES)
def test_qp_direct_matches_reference(ctx, name, N):
    """Method S (solveKKTSystem_Schur use_PCG=False, :441-446): the reference's
    np.linalg.solve on the dense S vs the GPU block-tridiagonal solve (k_btsolve)."""
    d = golden(f"qp_{name}_N{N}.npz")
    m = arm_model(name)
    ctx.set_model(m)
    ctx.set_cost_quadratic(*quad_cost_arrays(m.n))
    r = ctx.qp_batch(d["x"][None], d["u"][None], N, float(d["dt"]), float(d["rho"]), "S")
    assert _rel(r["S_diag"][0], d["S_diag"]) < 1e-11
    assert _rel(r["gamma"][0], d["gamma"]) < 1e-11
    assert int(r["pcg_iters"][0]) == 0
    nz = r["dxul"][0].size - d["lam_direct"].size
    assert _rel(r["dxul"][0][nz:], d["lam_direct"]) < 1e-9
    assert _rel(r["dxul"][0], d["dxul_direct"]) < 1e-9


def test_pcg_batch_matches_singles(ctx):
    """Problems are independent: a batch equals the problems solved one by one (bitwise)."""
    d = golden("qp_arm3_N32.npz")
    rng = np.random.default_rng(0)
    B = 33
    scale = rng.uniform(0.5, 2.0, B)
    Sd = d["S_diag"][None] * scale[:, None, None, None]
    Sl = d["S_lo"][None] * scale[:, None, None, None]
    g = d["gamma"][None] * rng.uniform(0.5, 2.0, (B, 1))
    lam, it, _, _, _ = ctx.pcg_batch(Sd, Sl, g, precond="SS", trace=False)
    for b in (0, 7, 32):
        l1, i1, _, _, _ = ctx.pcg_batch(Sd[b:b + 1], Sl[b:b + 1], g[b:b + 1], precond="SS", trace=False)
        assert i1[0] == it[b]
        assert np.array_equal(l1[0], lam[b])


def test_pcg_guess_and_edge_sizes(ctx):
    """Warm start (PCG.update_guess) and the smallest horizon N = 1."""
    d = golden("qp_arm2_N8.npz")
    lam, it, _, _, _ = ctx.pcg_batch(d["S_diag"][None], d["S_lo"][None], d["gamma"][None], precond="BJ")
    lam2, it2, _, _, _ = ctx.pcg_batch(d["S_diag"][None], d["S_lo"][None], d["gamma"][None], precond="BJ",
                                       guess=lam)
    assert it2[0] <= 1
    Sd = d["S_diag"][:1][None]
    lam1, it1, _, _, _ = ctx.pcg_batch(Sd, np.zeros((1, 1, 4, 4)), d["gamma"][:4][None], precond="SS")
    ref = np.linalg.solve(Sd[0, 0], d["gamma"][:4])
    assert np.allclose(lam1[0], ref, rtol=1e-9, atol=1e-12)
