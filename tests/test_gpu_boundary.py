"""GPU parity of the reference's QP-level solver methods on the drop-in (TrajoptMPCReference.py:118-455):
formKKTSystemBlocks, solveKKTSystem, solveKKTSystem_Schur, totalCost, totalHardConstraintViolation --
each called exactly as the reference's callers call it, against the reference's own recorded values:

  * the first QP of the reference's recorded SQP solves (tests/golden/sqp_*.npz, hard_*.npz: the QP at
    (x0, u0), xs = x0[:, 0], rho = rho_init = 1e-3; `dxul` row 0 is the reference's solveKKTSystem /
    solveKKTSystem_Schur output there) -- dxul within 1e-8 of max|dxul| (the PCG methods: the
    reference's truncated PCG iterate, with the iteration count exact);
  * the QP fixtures (tests/golden/qp_*.npz: the reference's g, c, A_k, B_k) for formKKTSystemBlocks --
    G and g bit for bit (the cost hooks are host arithmetic), C and c within 1e-12 (GPU dynamics);
  * the trace's first row (J, c at (x0, u0)) for totalCost (bit for bit) / totalHardConstraintViolation.
"""
import glob
import os

import numpy as np
import pytest

from conftest import ARM_N, GOLDEN, quad_cost_arrays

pytestmark = pytest.mark.gpu


def _arm_solver(name, N=None, hard=None):
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant,
                                         planar_arm_urdf)
    n = ARM_N[name]
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
    return TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(n)))


def _hard_solver(d):
    from trajoptmpcreference_amd import QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant
    N = d["x0"].shape[1]
    plant = URDFPlant(options={"path_to_urdf": str(d["urdf"])})
    con = TrajoptConstraint(1, 1, 1, N)
    con.set_torque_limits([float(d["ub"])], [float(d["lb"])], str(d["mode"]))
    return TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(1)), con)


def _parse(f):
    name, Ns, ss, method = os.path.basename(f)[4:-4].split("_")
    return name, int(Ns[1:]), method


SQP_FILES = sorted(glob.glob(os.path.join(GOLDEN, "sqp_*.npz")))


@pytest.mark.parametrize("f", SQP_FILES, ids=lambda f: os.path.basename(f))
def test_first_qp_matches_reference(f):
    """QP 0 of each recorded solve through the reference-named method its SQP calls (:598-605)."""
    name, N, method = _parse(f)
    d = np.load(f)
    solver = _arm_solver(name)
    x0, u0, dt = d["x0"], d["u0"], float(d["dt"])
    xs = x0[:, 0].copy()
    if method == "N":
        dxul = solver.solveKKTSystem(x0, u0, xs, N, dt, 1e-3)
    elif method == "S":
        dxul = solver.solveKKTSystem_Schur(x0, u0, xs, N, dt, 1e-3)    # use_PCG defaults to False (:361)
    else:
        dxul = solver.solveKKTSystem_Schur(x0, u0, xs, N, dt, 1e-3, True,
                                           {"preconditioner_type": method[4:], "exit_tolerance": 1e-6,
                                            "max_iter": 100})
        assert solver.n_inner_iter == int(d["pcg_iters"][0]), (solver.n_inner_iter, int(d["pcg_iters"][0]))
    ref = d["dxul"][0]
    assert dxul.shape == (ref.shape[0], 1)
    err = float(np.max(np.abs(dxul[:, 0] - ref))) / max(1.0, float(np.max(np.abs(ref))))
    assert err < 1e-8, err


HARD_AS = [f for f in sorted(glob.glob(os.path.join(GOLDEN, "hard_*_AS_*.npz")))]


@pytest.mark.parametrize("f", HARD_AS, ids=lambda f: os.path.basename(f))
def test_first_qp_hard_rows_match_reference(f):
    """QP 0 with the reference's active hard rows appended after each knot's dynamics rows (:238-248):
    dxul = [dxu; lambda] with lambda in the reference's row order (dynamics and hard multipliers
    interleaved by knot), against the reference's own dxul; formKKTSystemBlocks' C has the reference's
    row count (C_rows)."""
    d = np.load(f)
    method = os.path.basename(f)[:-4].split("_")[-1]
    solver = _hard_solver(d)
    x0, u0, dt = d["x0"], d["u0"], float(d["dt"])
    N = x0.shape[1]
    xs = x0[:, 0].copy()
    G, g, C, c = solver.formKKTSystemBlocks(x0, u0, xs, N, dt)
    assert C.shape[0] == int(d["C_rows"][0]) and c.shape == (C.shape[0], 1)
    if method == "N":
        dxul = solver.solveKKTSystem(x0, u0, xs, N, dt, 1e-3)
    elif method == "S":
        dxul = solver.solveKKTSystem_Schur(x0, u0, xs, N, dt, 1e-3)
    else:
        dxul = solver.solveKKTSystem_Schur(x0, u0, xs, N, dt, 1e-3, True, {"preconditioner_type": method[4:]})
        assert solver.n_inner_iter == int(d["pcg_iters"][0])
    ref = d["dxul"][0]
    ref = ref[~np.isnan(ref)]
    assert dxul.shape == (ref.shape[0], 1), (dxul.shape, ref.shape)
    err = float(np.max(np.abs(dxul[:, 0] - ref))) / max(1.0, float(np.max(np.abs(ref))))
    assert err < 1e-8, err
    # the KKT system formKKTSystemBlocks returns is the one dxul solves (method N: exactly up to rounding)
    if method in ("N", "S"):
        K = np.block([[G + 1e-3 * np.eye(G.shape[0]), C.T], [C, np.zeros((C.shape[0], C.shape[0]))]])
        res = np.max(np.abs(K @ dxul - np.vstack((g, c))))
        assert res < 1e-9, res


@pytest.mark.parametrize("name,N", [("arm2", 8), ("arm3", 32), ("arm6fix", 64)])
def test_form_kkt_system_blocks_matches_reference(name, N):
    d = np.load(os.path.join(GOLDEN, f"qp_{name}_N{N}.npz"))
    n = ARM_N[name]
    nx, nu = 2 * n, n
    solver = _arm_solver(name)
    x, u, dt = d["x"], d["u"], float(d["dt"])
    G, g, C, c = solver.formKKTSystemBlocks(x, u, x[:, 0].copy(), N, dt)
    nz = (nx + nu) * (N - 1) + nx
    assert G.shape == (nz, nz) and g.shape == (nz, 1) and C.shape == (nx * N, nz) and c.shape == (nx * N, 1)
    Q, QF, R, _ = quad_cost_arrays(n)
    Gref = np.zeros((nz, nz))
    for k in range(N - 1):
        s = k * (nx + nu)
        Gref[s:s + nx, s:s + nx] = Q
        Gref[s + nx:s + nx + nu, s + nx:s + nx + nu] = R
    Gref[nz - nx:, nz - nx:] = QF
    assert np.array_equal(G, Gref)
    assert np.array_equal(g[:, 0], d["g"])
    Cref = np.zeros((nx * N, nz))
    Cref[:nx, :nx] = np.eye(nx)
    for k in range(N - 1):
        s = k * (nx + nu)
        Cref[(k + 1) * nx:(k + 2) * nx, s:s + nx] = -d["A"][k]
        Cref[(k + 1) * nx:(k + 2) * nx, s + nx:s + nx + nu] = -d["B"][k]
        Cref[(k + 1) * nx:(k + 2) * nx, s + nx + nu:s + 2 * nx + nu] = np.eye(nx)
    assert float(np.max(np.abs(C - Cref))) < 1e-12 * max(1.0, float(np.max(np.abs(Cref))))
    assert float(np.max(np.abs(c[:, 0] - d["c"]))) < 1e-12 * max(1.0, float(np.max(np.abs(x))))


@pytest.mark.parametrize("f", SQP_FILES + HARD_AS, ids=os.path.basename)
def test_total_cost_and_violation_match_trace(f):
    """totalCost / totalHardConstraintViolation at (x0, u0) = the reference trace's first J and c (:541-542)
    (single-pass solves: with soft limits the recorded trace is the last outer pass's)."""
    d = np.load(f)
    if os.path.basename(f).startswith("sqp_"):
        name, N, _ = _parse(f)
        solver = _arm_solver(name)
    else:
        solver = _hard_solver(d)
        N = d["x0"].shape[1]
    x0, u0, dt = d["x0"], d["u0"], float(d["dt"])
    J = solver.totalCost(x0, u0, N)
    c = solver.totalHardConstraintViolation(x0, u0, x0[:, 0].copy(), N, dt)
    assert J == float(d["tr_J"][0]), (J, float(d["tr_J"][0]))
    assert abs(c - float(d["tr_c"][0])) <= 1e-12 * max(1.0, abs(float(d["tr_c"][0]))), (c, float(d["tr_c"][0]))
    cm = solver.totalHardConstraintViolation(x0, u0, x0[:, 0].copy(), N, dt, "MAX")
    assert cm <= c + 1e-15


def test_mpc_qp_n_method():
    """MPCSolverMethods.QP_N (TrajoptMPCReference.py:23): the horizon solves by method N equal method S's
    (the same KKT solution, the same direct path)."""
    from oracle import sqp as osqp
    from trajoptmpcreference_amd import MPCSolverMethods
    from conftest import arm_model
    m = arm_model("arm3")
    solver = _arm_solver("arm3")
    xs, us = zip(*[osqp.initial_problem(m, 16, 0.1, s) for s in range(3)])
    rn = solver.MPC_batch(np.array(xs), np.array(us), 16, 0.1, MPCSolverMethods.QP_N, {}, mpc_steps=2)
    rs = solver.MPC_batch(np.array(xs), np.array(us), 16, 0.1, MPCSolverMethods.QP_S, {}, mpc_steps=2)
    assert np.array_equal(rn["x_exec"], rs["x_exec"]) and np.array_equal(rn["exit_codes"], rs["exit_codes"])


@pytest.mark.parametrize("mode", ["QUADRATIC_PENALTY", "AUGMENTED_LAGRANGIAN"])
def test_soft_limit_qp_solves_the_dense_kkt(mode):
    """tmpc_qp_batch with soft limits (the jacobian terms of formKKTSystemBlocks :220-225, :255-259 formed on
    the device at the constraint objects' mu / lambda): solveKKTSystem_Schur's dxul solves the dense KKT
    system that formKKTSystemBlocks builds with the same hooks -- residual at rounding, for both soft modes,
    two limit kinds, and mu / lambda away from their defaults (TrajoptConstraint.py:138-166)."""
    from oracle import sqp as osqp
    from conftest import arm_model
    from trajoptmpcreference_amd import QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant, \
        planar_arm_urdf
    n, N, dt, rho = 3, 10, 0.1, 2e-3
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
    con = TrajoptConstraint(n, n, n, N)
    con.set_torque_limits([0.2] * n, [-0.2] * n, mode)
    con.set_joint_limits([0.5] * n, [-0.5] * n, mode)
    rng = np.random.default_rng(11)
    for box in (con.torque_limits, con.joint_limits):
        box.quadratic_penalty_mu[:] = rng.uniform(0.5, 5.0, box.quadratic_penalty_mu.shape)
        box.augmented_lagrangian_lambda[:] = rng.uniform(-0.3, 0.3, box.augmented_lagrangian_lambda.shape)
    solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(n)), con)
    x, u = osqp.initial_problem(arm_model("arm3"), N, dt, 21)
    u = u + rng.uniform(-0.6, 0.6, u.shape)   # torques outside +-0.2, joints outside +-0.5
    xs = x[:, 0].copy()
    G, g, C, c = solver.formKKTSystemBlocks(x, u, xs, N, dt)
    assert np.any(G[np.triu_indices_from(G, 1)] != 0)   # the soft terms' outer products are present
    Kk = np.block([[G + rho * np.eye(G.shape[0]), C.T], [C, np.zeros((C.shape[0], C.shape[0]))]])
    rhs = np.vstack((g, c))
    for dxul in (solver.solveKKTSystem_Schur(x, u, xs, N, dt, rho),
                 solver.solveKKTSystem(x, u, xs, N, dt, rho)):
        res = float(np.max(np.abs(Kk @ dxul - rhs)))
        assert res < 1e-9 * max(1.0, float(np.max(np.abs(rhs)))), res
