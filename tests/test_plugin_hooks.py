"""CPU: the TrajoptConstraint / BoxConstraint soft-constraint hooks of the drop-in
(trajoptmpcreference_amd/constraint.py) against the reference's own hook evaluations
(tests/golden/hooks_soft_arm1.npz, written by make_golden.py gen_soft_hooks from
/root/reference/TrajoptConstraint.py:53-166, 295-378): value_soft_constraints,
jacobian_soft_constraints, update_soft_constraint_constants (flag and the mu / lambda /
phi left behind), 1-link arm, torque and joint limits in QUADRATIC_PENALTY and
AUGMENTED_LAGRANGIAN.  Bit-for-bit: the hooks are a handful of IEEE operations in
the reference's order.  Plus the documented generalisations beyond what the
reference runs (several kinds at once, vector sizes) against oracle/soft.py."""
import numpy as np
import pytest

from conftest import golden

CASES = [(k, t) for k in ("torque", "joint") for t in ("QP", "AL")]
MODE = {"QP": "QUADRATIC_PENALTY", "AL": "AUGMENTED_LAGRANGIAN"}


def _constraint(kind, tag, d):
    from trajoptmpcreference_amd import TrajoptConstraint
    N = int(d["N"])
    con = TrajoptConstraint(1, 1, 1, N)
    getattr(con, f"set_{kind}_limits")([0.5], [-0.5], MODE[tag])
    box = getattr(con, f"{kind}_limits")
    pre = f"{kind}_{tag}_"
    T = d[pre + "mu0"].shape[1]          # the reference's knots (joint limits: N - 1)
    box.quadratic_penalty_mu[:, :T] = d[pre + "mu0"]
    box.augmented_lagrangian_lambda[:, :T] = d[pre + "lam0"]
    box.augmented_lagrangian_phi[:, :T] = d[pre + "phi0"]
    return con, box, pre, T


@pytest.mark.parametrize("kind,tag", CASES, ids=[f"{k}-{t}" for k, t in CASES])
def test_soft_value_and_jacobian_match_reference(kind, tag):
    d = golden("hooks_soft_arm1.npz")
    con, _, pre, _ = _constraint(kind, tag, d)
    for i in range(len(d[pre + "k"])):
        xk, uk, k = d[pre + "xk"][i], d[pre + "uk"][i], int(d[pre + "k"][i])
        v = con.value_soft_constraints(xk, uk, k)
        assert float(np.asarray(v).reshape(-1)[0]) == d[pre + "value"][i], (i, v, d[pre + "value"][i])
        j = con.jacobian_soft_constraints(xk, uk, k)
        assert j.shape == (3, 1)
        assert np.array_equal(j[:, 0], d[pre + "jac"][i]), (i, j[:, 0], d[pre + "jac"][i])


@pytest.mark.parametrize("kind,tag", CASES, ids=[f"{k}-{t}" for k, t in CASES])
def test_soft_update_matches_reference(kind, tag):
    d = golden("hooks_soft_arm1.npz")
    con, box, pre, T = _constraint(kind, tag, d)
    for r in range(len(d[pre + "upd_flag"])):
        flag = con.update_soft_constraint_constants(d[pre + "upd_x"][r], d[pre + "upd_u"][r])
        assert flag == bool(d[pre + "upd_flag"][r]), r
        assert np.array_equal(box.quadratic_penalty_mu[:, :T], d[pre + "upd_mu"][r]), r
        assert np.array_equal(box.augmented_lagrangian_lambda[:, :T], d[pre + "upd_lam"][r]), r
        assert np.array_equal(box.augmented_lagrangian_phi[:, :T], d[pre + "upd_phi"][r]), r


def test_box_update_hook_on_its_slice():
    """BoxConstraint.update_soft_constraint_constants (:138-166) called directly with the limited slice."""
    from trajoptmpcreference_amd import BoxConstraint
    d = golden("hooks_soft_arm1.npz")
    b = BoxConstraint(1, int(d["N"]) - 1, [0.5], [-0.5], "AUGMENTED_LAGRANGIAN")
    b.quadratic_penalty_mu[:] = d["torque_AL_mu0"]
    b.augmented_lagrangian_lambda[:] = d["torque_AL_lam0"]
    b.augmented_lagrangian_phi[:] = d["torque_AL_phi0"]
    assert b.update_soft_constraint_constants(d["torque_AL_upd_u"][0]) == bool(d["torque_AL_upd_flag"][0])
    assert np.array_equal(b.quadratic_penalty_mu, d["torque_AL_upd_mu"][0])
    assert np.array_equal(b.augmented_lagrangian_lambda, d["torque_AL_upd_lam"][0])


def test_soft_hooks_vector_and_several_kinds_match_oracle():
    """n = 3, torque + joint + velocity limits at once (what the reference cannot run):
    the value is the sum over the kinds, the jacobian the sum of the per-kind columns, the update
    runs for every kind -- the semantics of oracle/soft.py, which the GPU kernels follow."""
    from oracle import soft as osoft
    from trajoptmpcreference_amd import TrajoptConstraint
    n, N = 3, 6
    rng = np.random.default_rng(5)
    con = TrajoptConstraint(n, n, n, N)
    con.set_torque_limits([0.4] * n, [-0.3] * n, "AUGMENTED_LAGRANGIAN")
    con.set_joint_limits([0.7] * n, [-0.6] * n, "QUADRATIC_PENALTY")
    con.set_velocity_limits([0.5] * n, [-0.5] * n, "AUGMENTED_LAGRANGIAN")
    lims = []
    for kind, lb, ub in (("joint", -0.6, 0.7), ("velocity", -0.5, 0.5), ("torque", -0.3, 0.4)):
        c = getattr(con, f"{kind}_limits")
        lim = osoft.SoftLimit(kind, n, N, lb, ub, c.mode)
        c.augmented_lagrangian_lambda[:] = rng.uniform(-1, 1, c.augmented_lagrangian_lambda.shape)
        lim.lam[:] = c.augmented_lagrangian_lambda
        lims.append(lim)
    oc = osoft.SoftConstraints(lims)
    X = rng.uniform(-1, 1, (2 * n, N))
    U = rng.uniform(-1, 1, (n, N - 1))
    for k in range(N):
        uk = U[:, k] if k < N - 1 else None
        assert con.value_soft_constraints(X[:, k], uk, k) == pytest.approx(oc.value(X[:, k], uk, k, N), rel=1e-15)
        j = con.jacobian_soft_constraints(X[:, k], uk, k)[:, 0]
        jo = sum(oc.jacobians(X[:, k], uk, k, N, 3 * n))
        assert np.allclose(j, jo, rtol=1e-15, atol=0)
    assert con.update_soft_constraint_constants(X, U) == oc.update(X, U)
    for c, lim in zip((con.joint_limits, con.velocity_limits, con.torque_limits), lims):
        assert np.array_equal(c.quadratic_penalty_mu, lim.mu)
        assert np.array_equal(c.augmented_lagrangian_lambda, lim.lam)
        assert np.array_equal(c.augmented_lagrangian_phi, lim.phi)


def test_soft_hooks_without_soft_limits():
    from trajoptmpcreference_amd import TrajoptConstraint
    con = TrajoptConstraint(1, 1, 1, 5)
    assert con.value_soft_constraints(np.zeros(2), np.zeros(1), 0) == 0
    assert con.jacobian_soft_constraints(np.zeros(2), np.zeros(1), 0) is None
    con.set_torque_limits([1.0], [-1.0], "ACTIVE_SET")      # hard limits have no soft terms
    assert con.value_soft_constraints(np.zeros(2), np.array([3.0]), 0) == 0
    assert con.jacobian_soft_constraints(np.zeros(2), np.array([3.0]), 0) is None


def test_reference_hooks_three_kinds_match_reference():
    """TrajoptConstraint.reference_hooks = True against the reference's own hooks with three soft kinds
    at once (tests/golden/hooks_soft_multi_arm1.npz, make_golden.py gen_soft_hooks_multi): the value,
    the vstacked jacobian, max_soft_constraint_value, and the short-circuit update (later kinds left
    untouched once a kind returns False), bit for bit.  The default (device) semantics differ exactly
    there: velocity limits on qd, summed jacobians, every kind updated."""
    from trajoptmpcreference_amd import TrajoptConstraint
    d = golden("hooks_soft_multi_arm1.npz")
    N = int(d["N"])

    def make(ref):
        con = TrajoptConstraint(1, 1, 1, N)
        con.reference_hooks = ref
        con.set_joint_limits([0.5], [-0.5], "QUADRATIC_PENALTY")
        con.set_velocity_limits([0.4], [-0.4], "AUGMENTED_LAGRANGIAN")
        con.set_torque_limits([0.3], [-0.3], "AUGMENTED_LAGRANGIAN")
        for kind in ("joint", "velocity", "torque"):
            box = getattr(con, f"{kind}_limits")
            T = d[f"{kind}_mu0"].shape[1]
            box.quadratic_penalty_mu[:, :T] = d[f"{kind}_mu0"]
            box.augmented_lagrangian_lambda[:, :T] = d[f"{kind}_lam0"]
            box.augmented_lagrangian_phi[:, :T] = d[f"{kind}_phi0"]
        return con

    con = make(True)
    for i in range(len(d["k"])):
        xk, uk, k = d["xk"][i], d["uk"][i], int(d["k"][i])
        assert float(np.asarray(con.value_soft_constraints(xk, uk, k)).reshape(-1)[0]) == d["value"][i], i
        assert np.array_equal(con.jacobian_soft_constraints(xk, uk, k), d["jac"][i]), i
    for r in range(len(d["upd_flag"])):
        X, U = d["upd_x"][r], d["upd_u"][r]
        assert con.max_soft_constraint_value(X, U) == d["max_value"][r], r
        assert con.update_soft_constraint_constants(X, U) == bool(d["upd_flag"][r]), r
        for kind in ("joint", "velocity", "torque"):
            box = getattr(con, f"{kind}_limits")
            T = d[f"{kind}_mu0"].shape[1]
            assert np.array_equal(box.quadratic_penalty_mu[:, :T], d[f"upd_{kind}_mu"][r]), (r, kind)
            assert np.array_equal(box.augmented_lagrangian_lambda[:, :T], d[f"upd_{kind}_lam"][r]), (r, kind)
            assert np.array_equal(box.augmented_lagrangian_phi[:, :T], d[f"upd_{kind}_phi"][r]), (r, kind)
    # the device semantics are a different function on the same inputs
    dev = make(False)
    xk, uk, k = d["xk"][0], d["uk"][0], int(d["k"][0])
    assert dev.jacobian_soft_constraints(xk, uk, k).shape == (3, 1)
    assert d["jac"][0].shape == (9, 1)
