"""CPU: pin oracle/eecost.py (the restatement of the reference's end-effector
cost UrdfCost, TrajoptCost.py:371-569, and the RBDReference EE kinematics it
calls, RBDReference.py:123-387) to the reference's own outputs:

  * ee_arm2_points.npz   value / gradient / hessian / EE position / Jacobian /
                         jacobian_tot_state at 24 random arm2 states (running
                         and terminal knots, QF_start = 20);
  * ee_sqp_arm2_N10_*.npz  full SQP solves of examples/twolinks.py's
                         configuration (the one data/4 and data/3 were recorded
                         with), PCG-SS and S;
  * ee_arm2_recorded.npz  final_traj / final_input CSVs of the recorded runs
                         data/4 and data/3.

Integer outputs (exit code, SQP iterations, PCG iteration counts, line-search
alpha sequence) must be identical; floating point within the stated tolerances.
"""
import numpy as np
import pytest

from conftest import arm_model, golden
from oracle import eecost
from oracle import sqp as osqp


def _rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b)))) / max(1.0, float(np.max(np.abs(b))))


def _cost(xg, QF_start=None):
    return eecost.UrdfCost(arm_model("arm2"), np.eye(4), 100.0 * np.eye(4), 0.1 * np.eye(2), xg, QF_start)


def test_ee_kinematics_and_cost_hooks_match_reference():
    d = golden("ee_arm2_points.npz")
    m = arm_model("arm2")
    cost = _cost(d["xg"], int(d["QF_start"]))
    for i, x in enumerate(d["X"]):
        term = bool(d["terminal"][i])
        u = None if term else d["U"][i]
        k = int(d["k"][i])
        q, qd = x[:2], x[2:]
        assert np.allclose(eecost.end_effector_position(m, q), d["pos"][i], rtol=0, atol=1e-12)
        assert np.allclose(eecost.jacobian(m, q), d["J"][i], rtol=0, atol=1e-12)
        assert np.allclose(eecost.jacobian_tot_state(m, q, qd), d["Jtot"][i], rtol=0, atol=1e-12)
        assert np.allclose(cost.delta_x(x), d["dx"][i], rtol=0, atol=1e-12)
        assert abs(cost.value(x, u, k) - d["value"][i]) <= 1e-12 * max(1.0, abs(d["value"][i]))
        nz = 4 if term else 6
        assert _rel(cost.gradient(x, u, k), d["grad"][i][:nz]) < 1e-12
        assert _rel(cost.hessian(term, k, x), d["hess"][i][:nz, :nz]) < 1e-12


def test_ee_cost_rejects_non_2link_models():
    with pytest.raises(ValueError, match="2-link"):
        eecost.UrdfCost(arm_model("arm3"), np.eye(6), np.eye(6), np.eye(3), np.zeros(6))


@pytest.mark.parametrize("tag,method", [("d4", "PCG-SS"), ("d3", "PCG-SS"), ("d4", "S")])
def test_ee_sqp_matches_reference(tag, method):
    d = golden(f"ee_sqp_arm2_N10_{tag}_{method}.npz")
    N, dt = 10, float(d["dt"])
    cost = _cost(d["xg"])
    r = osqp.sqp(arm_model("arm2"), cost, d["x0"], d["u0"], N, dt, method,
                 {"expected_reduction_min_SQP_DDP": float(d["expected_reduction_min"])})
    assert r["exit_sqp"] == int(d["exit_sqp"])
    assert r["sqp_iter"] == int(d["sqp_iter"])
    if method != "S":
        assert list(r["pcg_iters"]) == list(d["pcg_iters"])
    alphas = [t["alpha"] for t in r["trace"]]
    assert np.array_equal(np.array(alphas, dtype=float), d["tr_alpha"])
    # truncated-PCG iterates: the difference is summation order inside PCG, carried
    # through 9 SQP iterations on data/3's configuration (2.0e-6 there)
    assert _rel(r["x"], d["x"]) < 1e-6
    assert _rel(r["u"], d["u"]) < 1e-6


@pytest.mark.parametrize("tag,xg", [("4", [-1.0, 1.5, 0.0, 0.0]), ("3", [-1.18, -1.58, 0.0, 0.0])])
def test_ee_sqp_reproduces_recorded_runs(tag, xg):
    """data/<tag>/final_traj.csv and final_input.csv: the reference authors' own
    recorded twolinks runs.  SURVEY F10 measured the reference itself reproducing
    them to 2.3e-7 (data/4) and 2.0e-6 (data/3)."""
    rec = golden("ee_arm2_recorded.npz")
    N = 10
    r = osqp.sqp(arm_model("arm2"), _cost(np.array(xg)), np.zeros((4, N)), np.zeros((2, N - 1)), N, 0.1, "PCG-SS",
                 {"expected_reduction_min_SQP_DDP": -100})
    # |x| reaches 4.7 on data/3; the reference run today is itself 2.0e-6 away from it
    assert np.max(np.abs(r["x"] - rec[f"d{tag}_final_traj"])) < 1e-5
    assert np.max(np.abs(r["u"] - rec[f"d{tag}_final_input"])) < 1e-5


def test_host_urdfcost_hooks_match_reference():
    """The drop-in's host UrdfCost (trajoptmpcreference_amd/cost.py) -- the plugin hooks
    callers evaluate themselves, e.g. exampleHelpers.py:101-111 -- against the same
    reference evaluations (no GPU needed: URDFPlant only parses the model)."""
    from trajoptmpcreference_amd import URDFPlant, UrdfCost, planar_arm_urdf
    d = golden("ee_arm2_points.npz")
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(2)})
    cost = UrdfCost(plant, np.eye(4), 100.0 * np.eye(4), 0.1 * np.eye(2), d["xg"], int(d["QF_start"]))
    for i, x in enumerate(d["X"]):
        term = bool(d["terminal"][i])
        u = None if term else d["U"][i]
        k = int(d["k"][i])
        nz = 4 if term else 6
        assert np.allclose(cost.delta_x(x), d["dx"][i], rtol=0, atol=1e-12)
        assert np.allclose(cost.jacobian_tot_state(x[:2], x[2:]), d["Jtot"][i], rtol=0, atol=1e-12)
        assert abs(cost.value(x, u, k, iter_1=1, iter_2=0, iter_3=2) - d["value"][i]) <= 1e-12 * max(1.0, abs(d["value"][i]))
        assert _rel(cost.gradient(x, u, k), d["grad"][i][:nz]) < 1e-12
        assert _rel(cost.hessian(x, u, k), d["hess"][i][:nz, :nz]) < 1e-12
    with pytest.raises(ValueError, match="2-link"):
        UrdfCost(URDFPlant(options={"path_to_urdf": planar_arm_urdf(3)}), np.eye(6), np.eye(6), np.eye(3),
                 np.zeros(6))
