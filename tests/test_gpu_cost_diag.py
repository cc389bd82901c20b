"""Bitwise equivalence checks of alternative kernel paths.

* The diagonal-QuadraticCost fast path (CostDev.diag: the cost products without their exact-zero
  terms, in the rollout cost, the line-search terms and the Riccati staging) against the dense form
  (TMPC_GENERIC_COST=1): the same values bit for bit, in fp64 and in fp32, on the BASELINE config 3
  workload (iLQR + augmented-Lagrangian torque limits) and on SQP PCG-SS.
* k_ilqr_soft_add's multi-pass form (TMPC_SOFT_ADD_GROUP) against its single pass."""
import numpy as np
import pytest

from conftest import arm_model, golden, quad_cost_arrays

pytestmark = pytest.mark.gpu


def _problems(name, N, seeds):
    from oracle import sqp as osqp
    m = arm_model(name)
    xs, us = zip(*[osqp.initial_problem(m, N, 0.1, int(s)) for s in seeds])
    return np.array(xs), np.array(us)


def _solve(monkeypatch, generic, prec, solver):
    from trajoptmpcreference_amd import QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant, \
        planar_arm_urdf
    monkeypatch.setenv("TMPC_GENERIC_COST", generic)
    d = golden("oracle_config3_arm6_N64_ilqr_al.npz")
    N = int(d["N"])
    lb, ub = float(d["lb"]), float(d["ub"])
    con = TrajoptConstraint(6, 6, 6, N)
    con.set_torque_limits([ub] * 6, [lb] * 6, "AUGMENTED_LAGRANGIAN")
    s = TrajoptMPCReference(URDFPlant(options={"path_to_urdf": planar_arm_urdf(6)}),
                            QuadraticCost(*quad_cost_arrays(6)), con)
    x, u = _problems("arm6fix", N, d["seeds"])
    opts = {"max_iter_softConstraints": int(d["max_iter_softConstraints"]),
            "max_iter_SQP_DDP": int(d["max_iter_SQP_DDP"]), "precision": prec}
    if solver == "ilqr":
        return s.iLQR_batch(x, u, N, 0.1, opts)
    return s.SQP_batch(x, u, N, 0.1, "PCG-SS", opts)


@pytest.mark.parametrize("prec,solver", [("fp64", "ilqr"), ("fp32", "ilqr"), ("fp64", "sqp")])
def test_diag_cost_path_is_bitwise_the_dense_one(monkeypatch, prec, solver):
    a = _solve(monkeypatch, "1", prec, solver)
    b = _solve(monkeypatch, "0", prec, solver)
    for key in ("x", "u", "exit_code" if solver == "ilqr" else "exit_sqp"):
        assert np.array_equal(np.asarray(a[key]), np.asarray(b[key])), key


def test_soft_add_multipass_is_bitwise_the_single_pass(monkeypatch):
    """k_ilqr_soft_add evaluates the trials' soft values in passes of TG trials (as many [N + 1] LDS rows
    as fit in 48 KB; one pass at the BASELINE sizes).  TMPC_SOFT_ADD_GROUP=2 forces 5 passes for the 9
    trials: the config-3 iLQR solve must be bit for bit the single-pass one (same terms, same knot-order
    sums, only the LDS rows reused)."""
    monkeypatch.delenv("TMPC_SOFT_ADD_GROUP", raising=False)
    a = _solve(monkeypatch, "0", "fp64", "ilqr")
    monkeypatch.setenv("TMPC_SOFT_ADD_GROUP", "2")
    b = _solve(monkeypatch, "0", "fp64", "ilqr")
    for key in ("x", "u", "exit_code", "iter"):
        assert np.array_equal(np.asarray(a[key]), np.asarray(b[key])), key
