"""The dense PCG restatement (oracle/dense.py, the operation order of tmpc_pcg_dense_batch) pinned to the
reference's own PCG (GBD-PCG-Python/PCG.py:66-111) on the reference's own Schur complements and
preconditioner matrices (tests/golden/qp_*.npz, written by make_golden.py from the reference): with the
reference's Pinv (the arbitrary-Pinv entry) and with the canonical block preconditioner (PCG.solve's own),
for 0 / J / BJ / SS and from the reference's warm start, the iteration count is the reference's exactly,
lambda within 1e-8 of max|lambda| (1e-5 unpreconditioned), the |nu| and ||b - A x|| traces within 1e-6
relative.  The GPU tests hold the kernel bit for bit to this restatement (test_gpu_pcg_dense.py)."""
import numpy as np
import pytest

from conftest import golden

CASES = [(n, p) for n in ("qp_arm2_N8", "qp_arm3_N32", "qp_arm6fix_N64") for p in ("J", "BJ", "SS", "0")]


def _system(d):
    from oracle import dense as od
    return od.from_blocks(d["S_diag"], d["S_lo"], d["S_up"]), np.asarray(d["gamma"], dtype=float).reshape(-1)


def _ref_pinv(d, ptype):
    from oracle import dense as od
    if ptype == "0":
        return np.identity(d["S_diag"].shape[0] * d["S_diag"].shape[1])
    return od.from_blocks(d[f"P_{ptype}_diag"], d[f"P_{ptype}_lo"], d[f"P_{ptype}_up"])


def _check(d, key, x, it, tn, tr, ptype):
    assert it == int(d[f"iters_{key}"]), (key, it, int(d[f"iters_{key}"]))
    ref = np.asarray(d[f"lam_{key}"]).reshape(-1)
    tol = 1e-5 if ptype == "0" else 1e-8
    assert float(np.max(np.abs(x - ref))) <= tol * max(1.0, float(np.max(np.abs(ref))))
    if ptype != "0":   # plain CG's traces are rounding-chaotic after a few iterations
        m = max(1, it - 3)
        assert np.allclose(tn[:m], d[f"trace_nu_{key}"][:m], rtol=1e-6, atol=0)
        if f"trace_res_{key}" in d:
            assert np.allclose(tr[:m], d[f"trace_res_{key}"][:m], rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("name,ptype", CASES, ids=[f"{n}-{p}" for n, p in CASES])
def test_dense_pcg_with_the_references_pinv(name, ptype):
    from oracle import dense as od
    d = golden(f"{name}.npz")
    S, g = _system(d)
    x, it, tn, tr = od.pcg(S, g, _ref_pinv(d, ptype))
    _check(d, ptype, x, it, tn, tr, ptype)


@pytest.mark.parametrize("name,ptype", CASES, ids=[f"{n}-{p}" for n, p in CASES])
def test_dense_pcg_with_the_canonical_block_preconditioner(name, ptype):
    from oracle import dense as od
    d = golden(f"{name}.npz")
    S, g = _system(d)
    nx = d["S_diag"].shape[1]
    P = od.block_pinv(S, nx, ptype)
    if ptype in ("BJ", "SS"):
        assert float(np.max(np.abs(P - _ref_pinv(d, ptype)))) <= 1e-12 * float(np.max(np.abs(P)))
    x, it, tn, tr = od.pcg(S, g, P)
    _check(d, ptype, x, it, tn, tr, ptype)


@pytest.mark.parametrize("name", ["qp_arm2_N8", "qp_arm3_N32", "qp_arm6fix_N64"])
@pytest.mark.parametrize("ptype", ["BJ", "SS"])
def test_dense_pcg_warm_start(name, ptype):
    from oracle import dense as od
    d = golden(f"{name}.npz")
    S, g = _system(d)
    x, it, tn, tr = od.pcg(S, g, _ref_pinv(d, ptype), guess=d["guess"])
    _check(d, f"{ptype}_guess", x, it, tn, tr, ptype)
