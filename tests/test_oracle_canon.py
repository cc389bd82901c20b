"""The canonical-order PCG restatement (oracle/canon.c, the operation order of the GPU's fused QP kernel)
pinned to the reference's own PCG (GBD-PCG-Python/PCG.py:66-212) on the reference's own Schur
complements (tests/golden/qp_*.npz, written by make_golden.py from the reference): for every
preconditioner the iteration count is the reference's exactly, lambda within 1e-8 of max|lambda|
(1e-5 without a preconditioner: plain CG on cond(S) ~ 1e6 amplifies the order's last bits), the |nu| trace within 1e-6 relative until the
last iterations, and the block inverses (BJ / SS preconditioner blocks) within 1e-12.  The GPU tests
then hold the kernel bit for bit to this restatement on identical inputs (test_gpu_sqp.py,
test_gpu_pcg.py)."""
import numpy as np
import pytest

from conftest import golden


@pytest.fixture(scope="module")
def canon():
    from oracle import canon as c
    try:
        c._lib()
    except FileNotFoundError:
        import subprocess
        import os
        subprocess.run(["make", "-C", os.path.dirname(c.__file__)], check=True)
    return c


@pytest.mark.parametrize("rpl", [1, 2])
@pytest.mark.parametrize("name", ["qp_arm2_N8", "qp_arm3_N32", "qp_arm6fix_N64"])
@pytest.mark.parametrize("ptype", ["J", "BJ", "SS", "0"])
def test_canonical_pcg_counts_match_reference(canon, name, ptype, rpl):
    """Both lane layouts of the kernel (one row of S per lane; two -- the register instance past 768
    rows and the HBM-row GM instance) take the reference's counts on its own S."""
    d = golden(f"{name}.npz")
    lam, it, tn = canon.pcg(d["S_diag"], d["S_lo"], d["gamma"], ptype, rpl=rpl)
    assert it == int(d[f"iters_{ptype}"])
    ref = d[f"lam_{ptype}"]
    # unpreconditioned CG ('0') on cond(S) ~ 1e6 amplifies the order's rounding in its truncated iterate
    tol = 1e-5 if ptype == "0" else 1e-8
    assert float(np.max(np.abs(lam - ref))) <= tol * max(1.0, float(np.max(np.abs(ref))))
    if ptype != "0":   # plain CG's |nu| trace is rounding-chaotic after a few iterations (counts still agree)
        ref_nu = d[f"trace_nu_{ptype}"][:it + 1]
        m = max(1, it - 3)   # the last iterations' |nu| is summation-order noise near the exit
        assert np.allclose(tn[:m], ref_nu[:m], rtol=1e-6, atol=0)


@pytest.mark.parametrize("name", ["qp_arm2_N8", "qp_arm3_N32", "qp_arm6fix_N64"])
def test_canonical_block_inverse(canon, name):
    d = golden(f"{name}.npz")
    P = canon.block_inverse(d["S_diag"])
    ref = d["P_BJ_diag"]
    assert float(np.max(np.abs(P - ref))) <= 1e-12 * float(np.max(np.abs(ref)))


def test_canonical_layouts_and_warm_start(canon):
    """The two layouts are different operation orders (their lambdas differ in the last bits), the
    warm start from the solution itself exits at once, and sizes past the layout's 1024 lanes raise."""
    d = golden("qp_arm6fix_N64.npz")
    l1, i1, _ = canon.pcg(d["S_diag"], d["S_lo"], d["gamma"], "SS", rpl=1)
    l2, i2, _ = canon.pcg(d["S_diag"], d["S_lo"], d["gamma"], "SS", rpl=2)
    assert i1 == i2 and not np.array_equal(l1, l2)
    assert float(np.max(np.abs(l1 - l2))) < 1e-8 * float(np.max(np.abs(l1)))
    l3, i3, _ = canon.pcg(d["S_diag"], d["S_lo"], d["gamma"], "SS", rpl=2, guess=l2, tol=1e-3)
    assert i3 <= 2
    assert canon.qp_rpl(64, 12) == 1 and canon.qp_rpl(80, 12) == 2 and canon.qp_rpl(128, 12) == 2
    assert canon.qp_rpl(8, 6, gm_min_rows=1) == 2
    N, nx = 86, 12   # 1032 rows, 516 lanes at rpl 2; 1032 > 1024 lanes at rpl 1
    Sd = np.tile(-np.eye(nx), (N, 1, 1))
    with pytest.raises(ValueError):
        canon.pcg(Sd, np.zeros((N - 1, nx, nx)), np.ones(N * nx), "SS", rpl=1)
    lam, it, _ = canon.pcg(Sd, np.zeros((N - 1, nx, nx)), np.ones(N * nx), "SS", rpl=2)
    assert it == 1 and np.array_equal(lam, -np.ones(N * nx))
