"""GPU parity: soft box limits (QUADRATIC_PENALTY / AUGMENTED_LAGRANGIAN) and the
augmented-Lagrangian outer loop (TrajoptMPCReference.py:483-508,
TrajoptConstraint.py:53-166) through the TrajoptMPCReference drop-in.

* Against the reference's own solves (tests/golden/soft_*.npz, 1-link arm with
  torque limits -- the only box-constraint configuration the reference's code
  runs): exit codes, outer / SQP / line-search iteration counts and
  the alpha path identical; trajectories and merit terms at rtol 1e-7; the final
  mu / lambda / phi stored back into the BoxConstraint object.
* Against the oracle's vector semantics (oracle/soft.py) for n > 1 and several
  limit types at once (parity unpinned by the reference, which cannot run them).
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, arm_model, quad_cost_arrays

pytestmark = pytest.mark.gpu

SOFT_FILES = sorted(glob.glob(os.path.join(GOLDEN, "soft_*.npz")))


@pytest.mark.parametrize("f", SOFT_FILES, ids=lambda f: os.path.basename(f))
def test_soft_sqp_matches_reference(f):
    from trajoptmpcreference_amd import QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant
    d = np.load(f)
    N = d["x0"].shape[1]
    method = os.path.basename(f)[:-4].split("_")[-1]
    plant = URDFPlant(options={"path_to_urdf": str(d["urdf"])})
    con = TrajoptConstraint(1, 1, 1, N)
    con.set_torque_limits([float(d["ub"])], [float(d["lb"])], str(d["mode"]))
    solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(1)), con)
    x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(d["x0"], d["u0"], N, float(d["dt"]), method, {})
    assert (exit_sqp, exit_soft, outer_iter, sqp_iter) == (
        int(d["exit_sqp"]), int(d["exit_soft"]), int(d["outer_iter"]), int(d["sqp_iter"]))
    tr = solver.trace
    assert [t["alpha"] for t in tr] == list(d["tr_alpha"])
    assert [t["outer_iteration"] for t in tr] == list(d["tr_outer_iteration"].astype(int))
    assert [t["line_search_iteration"] for t in tr] == list(d["tr_line_search_iteration"].astype(int))
    assert [t["succeeded_line_search"] for t in tr] == list(d["tr_succeeded_line_search"].astype(bool))
    for key in ("J", "c", "merit", "rho"):
        assert np.allclose([t[key] for t in tr], d["tr_" + key], rtol=1e-7, atol=1e-12), key
    assert np.allclose(x, d["x"], rtol=1e-7, atol=1e-10)
    assert np.allclose(u, d["u"], rtol=1e-7, atol=1e-10)
    tl = con.torque_limits
    assert np.array_equal(tl.quadratic_penalty_mu, d["mu"])
    assert np.allclose(tl.augmented_lagrangian_lambda, d["lam"], rtol=1e-7, atol=1e-10)
    assert np.array_equal(tl.augmented_lagrangian_phi, d["phi"])


def _oracle_soft(n, N, spec):
    from oracle.soft import SoftConstraints, SoftLimit
    lims = []
    for kind in ("joint", "velocity", "torque"):
        if kind in spec:
            lb, ub, mode = spec[kind]
            lims.append(SoftLimit(kind, n, N, lb, ub, mode))
    return SoftConstraints(lims), lims


CASES = [
    ("arm3", 16, 6, "PCG-SS", {"torque": ([-0.7] * 3, [0.7] * 3, "AUGMENTED_LAGRANGIAN")}),
    ("arm3", 16, 6, "S", {"torque": ([-2.0] * 3, [2.0] * 3, "QUADRATIC_PENALTY"),
                          "joint": ([-0.8] * 3, [0.8] * 3, "AUGMENTED_LAGRANGIAN")}),
    ("arm3", 12, 4, "PCG-BJ", {"velocity": ([-1.0] * 3, [1.0] * 3, "QUADRATIC_PENALTY"),
                               "torque": ([-1.5] * 3, [1.5] * 3, "AUGMENTED_LAGRANGIAN")}),
    ("arm6fix", 32, 2, "PCG-SS", {"torque": ([-0.3] * 6, [0.3] * 6, "AUGMENTED_LAGRANGIAN")}),
]


@pytest.mark.parametrize("name,N,B,method,spec", CASES, ids=[f"{c[0]}-N{c[1]}-{c[3]}-{'+'.join(c[4])}" for c in CASES])
def test_soft_batch_matches_oracle(name, N, B, method, spec):
    """Vector semantics (oracle/soft.py) for n > 1 and several limit types, problem by problem."""
    from oracle import sqp as osqp
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant,
                                         planar_arm_urdf)
    m = arm_model(name)
    n = m.n
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
    con = TrajoptConstraint(n, n, n, N)
    for kind, (lb, ub, mode) in spec.items():
        getattr(con, f"set_{kind}_limits")(ub, lb, mode)
    solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(n)), con)
    xs, us = zip(*[osqp.initial_problem(m, N, 0.1, 300 + i) for i in range(B)])
    r = solver.SQP_batch(np.array(xs), np.array(us), N, 0.1, method, {})
    mu_g, lam_g, phi_g = r["soft_state"]
    for i in range(B):
        soft, lims = _oracle_soft(n, N, spec)
        o = osqp.sqp(m, osqp.QuadCost(*quad_cost_arrays(n)), xs[i], us[i], N, 0.1, method, {}, soft)
        got = (int(r["exit_sqp"][i]), int(r["exit_soft"][i]), int(r["outer_iter"][i]), int(r["sqp_iter"][i]))
        assert got == (o["exit_sqp"], o["exit_soft"], o["outer_iter"], o["sqp_iter"]), (i, got)
        scale = max(1.0, float(np.max(np.abs(o["x"]))))
        assert float(np.max(np.abs(r["x"][i] - o["x"]))) < 1e-6 * scale
        for lim in lims:
            t = ("joint", "velocity", "torque").index(lim.kind)
            sl = slice(t * 2 * n, (t + 1) * 2 * n)
            assert np.array_equal(mu_g[i, :lim.T, sl].T, lim.mu)
            assert np.allclose(lam_g[i, :lim.T, sl].T, lim.lam, rtol=1e-6, atol=1e-9)
            assert np.array_equal(phi_g[i, :lim.T, sl].T, lim.phi)


def test_soft_state_persists_like_the_reference_object():
    """A second SQP call starts from the constants the first one left in the BoxConstraint
    (the reference mutates the object in place), on the GPU as in the oracle."""
    from oracle import sqp as osqp
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant,
                                         planar_arm_urdf)
    m = arm_model("arm3")
    N = 8
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(3)})
    con = TrajoptConstraint(3, 3, 3, N)
    con.set_torque_limits([1.0] * 3, [-1.0] * 3, "AUGMENTED_LAGRANGIAN")
    solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(3)), con)
    x0, u0 = osqp.initial_problem(m, N, 0.1, 11)
    soft, lims = _oracle_soft(3, N, {"torque": ([-1.0] * 3, [1.0] * 3, "AUGMENTED_LAGRANGIAN")})
    opts = {"max_iter_softConstraints": 3}
    for _ in range(2):
        res = solver.SQP(x0, u0, N, 0.1, "PCG-SS", dict(opts))
        o = osqp.sqp(m, osqp.QuadCost(*quad_cost_arrays(3)), x0, u0, N, 0.1, "PCG-SS", dict(opts), soft)
        assert (res[2], res[3], res[4], res[5]) == (o["exit_sqp"], o["exit_soft"], o["outer_iter"], o["sqp_iter"])
        assert np.array_equal(con.torque_limits.quadratic_penalty_mu, lims[0].mu)
        assert np.allclose(con.torque_limits.augmented_lagrangian_lambda, lims[0].lam, rtol=1e-6, atol=1e-9)
