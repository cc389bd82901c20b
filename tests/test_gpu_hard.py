"""GPU parity: hard box constraints (BoxConstraint ACTIVE_SET / FULL_SET) in the SQP
(TrajoptMPCReference.py:238-248, 273-294; TrajoptConstraint.py:53-130, 210-293).

* Against the reference's own solves (tests/golden/hard_*.npz: 1-link arm, torque
  limits -- the only size the reference's BoxConstraint runs): exit
  code, SQP iterations, per-QP PCG counts (with the reference's nx-aligned
  preconditioner blocks that the appended rows shift), the alpha path, the
  constraint-violation trace and the trajectories.  FULL_SET with PCG: the
  reference raises LinAlgError (singular S), the drop-in raises too.
* Against the oracle's elementwise vector semantics (oracle/hard.py) for n > 1 and
  two limit types at once: integers exact except the PCG counts, which are held to
  the spread two summation orders of the oracle itself show there (see the test).
* QP by QP (tmpc_qp_batch with the hard rows): at every iterate of the oracle's SQP
  the GPU's QP step and dynamics-row multipliers against the oracle's dense solve.
  This is the parity statement for runs whose SQP-level path is rounding-decided:
  after a full step, entries land exactly on a bound and whether the next QP holds
  them active is decided by the last bit (pendulum, iterate 3: u[8..10] = 7 - 8.9e-16,
  7, 7 + 8.9e-16), so two correct solvers may take different active sets from there.
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, arm_model, quad_cost_arrays

pytestmark = pytest.mark.gpu

HARD_FILES = sorted(glob.glob(os.path.join(GOLDEN, "hard_*.npz")))


@pytest.mark.parametrize("f", HARD_FILES, ids=lambda f: os.path.basename(f))
def test_hard_sqp_matches_reference(f):
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant,
                                         _native)
    d = np.load(f)
    N = d["x0"].shape[1]
    method = os.path.basename(f)[:-4].split("_")[-1]
    plant = URDFPlant(options={"path_to_urdf": str(d["urdf"])})
    con = TrajoptConstraint(1, 1, 1, N)
    con.set_torque_limits([float(d["ub"])], [float(d["lb"])], str(d["mode"]))
    solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(1)), con)
    opts = {} if np.isnan(float(d["erm"])) else {"expected_reduction_min_SQP_DDP": float(d["erm"])}
    if str(d["error"]):
        with pytest.raises(_native.NativeError, match="FULL_SET"):
            solver.SQP(d["x0"], d["u0"], N, float(d["dt"]), method, opts)
        return
    x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(d["x0"], d["u0"], N, float(d["dt"]), method, opts)
    assert (exit_sqp, sqp_iter) == (int(d["exit_sqp"]), int(d["sqp_iter"]))
    tr = solver.trace
    assert [t["alpha"] for t in tr] == list(d["tr_alpha"])
    assert [t["line_search_iteration"] for t in tr] == list(d["tr_line_search_iteration"].astype(int))
    if method.startswith("PCG"):
        assert [t["inner_iters"] for t in tr[1:]] == list(d["pcg_iters"])
    for key in ("J", "c", "merit"):
        assert np.allclose([t[key] for t in tr], d["tr_" + key], rtol=1e-7, atol=1e-12), key
    assert np.allclose(x, d["x"], rtol=1e-7, atol=1e-10)
    assert np.allclose(u, d["u"], rtol=1e-7, atol=1e-10)


CASES = [
    ("arm3", 12, 3, "PCG-SS", {"torque": (-0.3, 0.3, "ACTIVE_SET"), "velocity": (-0.6, 0.6, "ACTIVE_SET")}),
    ("arm3", 12, 3, "PCG-BJ", {"torque": (-0.3, 0.3, "ACTIVE_SET"), "velocity": (-0.6, 0.6, "ACTIVE_SET")}),
    ("arm3", 12, 3, "S", {"torque": (-0.3, 0.3, "ACTIVE_SET"), "velocity": (-0.6, 0.6, "ACTIVE_SET")}),
    ("arm3", 12, 2, "S", {"velocity": (-0.5, 0.5, "FULL_SET")}),
    ("arm2", 16, 3, "PCG-SS", {"torque": (-0.4, 0.4, "ACTIVE_SET")}),
]


@pytest.mark.parametrize("name,N,B,method,spec", CASES,
                         ids=[f"{c[0]}-N{c[1]}-{c[3]}-{'+'.join(c[4])}" for c in CASES])
def test_hard_batch_matches_oracle(name, N, B, method, spec):
    """Elementwise vector semantics (oracle/hard.py), problem by problem: exit code, SQP iterations,
    per-QP PCG counts and the number of active rows of every QP; trajectories at 1e-6."""
    from oracle import hard as ohard
    from oracle import sqp as osqp
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant,
                                         planar_arm_urdf)
    m = arm_model(name)
    n = m.n
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
    con = TrajoptConstraint(n, n, n, N)
    for kind, (lb, ub, mode) in spec.items():
        getattr(con, f"set_{kind}_limits")([ub] * n, [lb] * n, mode)
    solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(n)), con)
    xs, us = zip(*[osqp.initial_problem(m, N, 0.1, 400 + i) for i in range(B)])
    r = solver.SQP_batch(np.array(xs), np.array(us), N, 0.1, method, {})
    hard = ohard.HardConstraints([ohard.HardLimit(k, n, lb, ub, mode) for k, (lb, ub, mode) in spec.items()])
    for i in range(B):
        o = osqp.sqp(m, osqp.QuadCost(*quad_cost_arrays(n)), xs[i], us[i], N, 0.1, method, {}, hard=hard)
        got = (int(r["exit_sqp"][i]), int(r["sqp_iter"][i]))
        assert got == (o["exit_sqp"], o["sqp_iter"]), (i, got)
        nq = got[1] + (1 if got[0] == 3 else 0)
        if method.startswith("PCG"):
            # With active rows the last dim mod nx rows of S get no preconditioner rows (PCG.py:182):
            # CG with that singular preconditioner is rounding-sensitive.  Measured: the oracle itself,
            # with its two matrix-vector products summed in reversed column order, moves these counts by
            # up to 4 ([38, 91, 91, 81, 71] -> [38, 87, 91, 80, 71] for BJ seed 400).  So the counts of
            # these reference-unpinned vector cases are held to that spread; the pinned 1-link fixtures
            # above are exact.
            got_it = [int(v) for v in r["trace"]["pcg_iters"][i, 1:nq + 1]]
            assert len(got_it) == len(o["pcg_iters"]), i
            assert all(abs(a - b) <= 5 for a, b in zip(got_it, o["pcg_iters"])), (i, got_it, o["pcg_iters"])
        assert list(r["trace"]["alpha"][i, 1:nq + 1]) == [t["alpha"] for t in o["trace"][1:]], i
        scale = max(1.0, float(np.max(np.abs(o["x"]))))
        assert float(np.max(np.abs(r["x"][i] - o["x"]))) < 1e-5 * scale, i


def test_hard_constraints_reject_ilqr():
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant, _native,
                                         planar_arm_urdf)
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(2)})
    con = TrajoptConstraint(2, 2, 2, 8)
    con.set_torque_limits([1.0] * 2, [-1.0] * 2, "ACTIVE_SET")
    solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(2)), con)
    with pytest.raises(_native.NativeError, match="iLQR"):
        solver.iLQR(np.zeros((4, 8)), np.zeros((2, 7)), 8, 0.1, {})


def _dyn_rows(hard, x, u, N, nx):
    """indices of the dynamics / initial-state rows in the oracle's row order (oracle/hard.py kkt_dense)"""
    idx = list(range(nx))
    r = nx
    for k in range(N - 1):
        idx += list(range(r, r + nx))
        r += nx + len(hard.rows(x[:, k], u[:, k], k, N))
    return idx


QP_CASES = [
    ("pendulum", 20, "S", {"torque": (-7.0, 7.0, "ACTIVE_SET")}),
    ("pendulum", 20, "PCG-SS", {"torque": (-7.0, 7.0, "ACTIVE_SET")}),
    ("arm3", 12, "PCG-SS", {"torque": (-0.3, 0.3, "ACTIVE_SET"), "velocity": (-0.6, 0.6, "ACTIVE_SET")}),
    ("arm3", 12, "PCG-BJ", {"torque": (-0.3, 0.3, "ACTIVE_SET"), "velocity": (-0.6, 0.6, "ACTIVE_SET")}),
    ("arm3", 12, "S", {"velocity": (-0.5, 0.5, "FULL_SET")}),
    ("arm2", 16, "PCG-J", {"torque": (-0.4, 0.4, "ACTIVE_SET"), "joint": (-1.0, 1.0, "ACTIVE_SET")}),
]


@pytest.mark.parametrize("name,N,method,spec", QP_CASES,
                         ids=[f"{c[0]}-N{c[1]}-{c[2]}-{'+'.join(c[3])}" for c in QP_CASES])
def test_hard_qp_matches_oracle_at_every_iterate(name, N, method, spec):
    """All QPs of one oracle SQP run, batched as B problems on the GPU: the step dxu and the
    dynamics-row multipliers (1e-9 relative for the direct solve S; for PCG, as close to the exact
    QP solution as the oracle's own PCG answer, up to 10x), PCG counts within the oracle's own
    summation-order spread (+-5, see above; the pendulum's iterate 2, 7 active rows, is 41 vs 42)."""
    from oracle import hard as ohard
    from oracle import sqp as osqp
    from trajoptmpcreference_amd import (PendulumPlant, QuadraticCost, TrajoptConstraint, TrajoptMPCReference,
                                         URDFPlant, planar_arm_urdf)
    if name == "pendulum":
        plant = PendulumPlant()
        n = 1
        Q, QF, R, xg = np.diag([1.0, 1.0]), np.diag([100.0, 100.0]), np.diag([0.1]), np.array([3.14159, 0.0])
        x0, u0 = np.zeros((2, N)), np.zeros((1, N - 1))
        opts = {"expected_reduction_min_SQP_DDP": -100}
    else:
        m = arm_model(name)
        n = m.n
        plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
        Q, QF, R, xg = quad_cost_arrays(n)
        x0, u0 = osqp.initial_problem(m, N, 0.1, 430)
        opts = {}
    nx = 2 * n
    con = TrajoptConstraint(n, n, n, N)
    for kind, (lb, ub, mode) in spec.items():
        getattr(con, f"set_{kind}_limits")([ub] * n, [lb] * n, mode)
    solver = TrajoptMPCReference(plant, QuadraticCost(Q, QF, R, xg), con)
    hard = ohard.HardConstraints([ohard.HardLimit(k, n, lb, ub, mode) for k, (lb, ub, mode) in spec.items()])
    model = plant.model if name == "pendulum" else m
    o = osqp.sqp(model, osqp.QuadCost(Q, QF, R, xg), x0, u0, N, 0.1, method, dict(opts), hard=hard)
    its = o["iterates"]
    assert len(its) == len(o["dxul"]) >= 2
    full = dict(opts)
    solver.set_default_options(full)
    ctx = solver._context(full)
    xs = np.array([x for x, _, _ in its])
    us = np.array([u for _, u, _ in its])
    rho = np.array([r for _, _, r in its])
    xs[:, :, 0] = x0[:, 0]      # the SQP's xs: the QP's initial-state row is x_0 - xs
    r = ctx.qp_batch(xs, us, N, 0.1, rho, method, want_blocks=False)
    nz = (nx + n) * (N - 1) + nx
    oc = osqp.QuadCost(Q, QF, R, xg)
    o_opts = osqp.default_options(opts)
    for i, (x, u, rho_i) in enumerate(its):
        ref = o["dxul"][i]
        rows = _dyn_rows(hard, x, u, N, nx)
        lam_ref = ref[nz:][rows]
        got = r["dxul"][i]
        if method != "S":
            assert abs(int(r["pcg_iters"][i]) - o["pcg_iters"][i]) <= 5, (i, int(r["pcg_iters"][i]),
                                                                               o["pcg_iters"][i])
        sc = max(1.0, float(np.max(np.abs(ref[:nz]))))
        sl = max(1.0, float(np.max(np.abs(lam_ref))))
        if method == "S":
            assert float(np.max(np.abs(got[:nz] - ref[:nz]))) < 1e-9 * sc, i
            assert float(np.max(np.abs(got[nz:] - lam_ref))) < 1e-9 * sl, i
            continue
        # PCG stops at |nu| < tol: its answer is as far from the exact QP solution as the tolerance
        # leaves it.  The GPU's solution must be as close to the exact one (the direct dense solve)
        # as the oracle's own PCG solution is, up to 10x.
        G, g, Cm, cc = ohard.kkt_dense(model, oc, x, u, x0[:, 0], N, 0.1, hard)
        ex, _, _ = ohard.solve_qp_dense(G, g, Cm, cc, rho_i, "S", o_opts, nx)
        e_ref = float(np.max(np.abs(ref[:nz] - ex[:nz])))
        e_got = float(np.max(np.abs(got[:nz] - ex[:nz])))
        assert e_got <= 10 * e_ref + 1e-9 * sc, (i, e_got, e_ref)
        el_ref = float(np.max(np.abs(lam_ref - ex[nz:][rows])))
        el_got = float(np.max(np.abs(got[nz:] - ex[nz:][rows])))
        assert el_got <= 10 * el_ref + 1e-9 * sl, (i, el_got, el_ref)


def test_hard_qp_rejects_blocks():
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant, _native,
                                         planar_arm_urdf)
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(2)})
    con = TrajoptConstraint(2, 2, 2, 8)
    con.set_torque_limits([1.0] * 2, [-1.0] * 2, "ACTIVE_SET")
    solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(2)), con)
    opts = {}
    solver.set_default_options(opts)
    ctx = solver._context(opts)
    with pytest.raises(_native.NativeError, match="NULL"):
        ctx.qp_batch(np.zeros((1, 4, 8)), np.zeros((1, 2, 7)), 8, 0.1, 0.001, "PCG-SS", want_blocks=True)
