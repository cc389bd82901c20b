"""Wide models: 8..12 joints (RBDReference.py:399-930 is generic in n).  The runtime-model
(ModelRef) dynamics -- forward dynamics, M^-1, the RNEA gradient, the Euler step and its Jacobians -- and
the SQP (TrajoptMPCReference.py:510-760) with the fused QP (one or two rows of S per lane) on generated
planar chains of 8, 9, 10 and 12 joints, against the oracle:
  * dynamics at 1e-12 of max|ref| (test_gpu_dynamics' bound);
  * SQP: exit code, SQP iterations, the alpha path and every QP's PCG count identical to the oracle's run
    (oracle/sqp.py), trajectories within 1e-6; every QP of the GPU's own run replayed at its own iterate
    with the canonical-order PCG (oracle/canon.c) on that QP's S: count and lambda bit for bit;
  * iLQR (the VALU Riccati sweep, the plain rollout) against oracle/ilqr.py: converged cost and trajectories,
    and every iteration replayed at the GPU's own iterate (test_gpu_ilqr._replay);
  * what a wide model does not run (box limits, the precision modes, the MPC loop, more than 1024 Schur
    rows for the SQP) is refused with a message naming the limit."""
import numpy as np
import pytest

from conftest import quad_cost_arrays, replay_qp_counts

pytestmark = pytest.mark.gpu


def _model(n):
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    return parse_urdf(planar_arm_urdf(n))


def _solver(n, con=None):
    from trajoptmpcreference_amd import QuadraticCost, TrajoptMPCReference, URDFPlant, planar_arm_urdf
    return TrajoptMPCReference(URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)}),
                               QuadraticCost(*quad_cost_arrays(n)), con)


def _close(a, b, tol=1e-12):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    assert float(np.max(np.abs(a - b))) <= tol * max(1.0, float(np.max(np.abs(b))))


@pytest.mark.parametrize("n", [8, 9, 12])
def test_wide_dynamics_match_oracle(ctx, n):
    from oracle import rbd
    m = _model(n)
    ctx.set_model(m)
    rng = np.random.default_rng(40 + n)
    K = 129
    x = np.hstack([rng.uniform(-np.pi, np.pi, (K, n)), rng.uniform(-3, 3, (K, n))])
    u = rng.uniform(-2, 2, (K, n))
    xn, qdd, Mi = ctx.fd_batch(x, u, 0.05)
    _close(qdd, rbd.forward_dynamics(m, x, u))
    _close(Mi, rbd.minv(m, x[:, :n]))
    _close(xn, rbd.euler(m, x, u, 0.05))
    A, B, _ = ctx.fd_grad_batch(x, u, 0.05)
    Ar, Br = rbd.euler_gradient(m, x, u, 0.05)
    _close(A, Ar)
    _close(B, Br)


CASES = [(9, 8, "PCG-SS", 900), (9, 12, "PCG-J", 901), (9, 10, "S", 902), (8, 16, "PCG-BJ", 903),
         (10, 20, "PCG-SS", 904), (12, 40, "PCG-SS", 905)]


@pytest.mark.parametrize("n,N,method,seed", CASES, ids=[f"n{c[0]}-N{c[1]}-{c[2]}" for c in CASES])
def test_wide_sqp_matches_oracle(n, N, method, seed):
    from oracle import sqp as osqp
    m = _model(n)
    x0, u0 = osqp.initial_problem(m, N, 0.1, seed)
    solver = _solver(n)
    r = solver.SQP_batch(x0[None], u0[None], N, 0.1, method, {})
    o = osqp.sqp(m, osqp.QuadCost(*quad_cost_arrays(n)), x0, u0, N, 0.1, method)
    ex, it = int(r["exit_sqp"][0]), int(r["sqp_iter"][0])
    assert (ex, it) == (o["exit_sqp"], o["sqp_iter"]), ((ex, it), (o["exit_sqp"], o["sqp_iter"]))
    nq = it + (1 if ex == 3 else 0)
    tr = r["trace"]
    assert [float(v) for v in tr["alpha"][0, 1:it + 1]] == [float(t["alpha"]) for t in o["trace"][1:it + 1]]
    counts = [int(v) for v in tr["pcg_iters"][0, 1:nq + 1]]
    if method != "S":
        assert counts == list(o["pcg_iters"][:nq]), (counts, o["pcg_iters"])
    scale = max(1.0, float(np.max(np.abs(o["x"]))))
    assert float(np.max(np.abs(r["x"][0] - o["x"]))) < 1e-6 * scale
    if method.startswith("PCG"):
        succ = [bool(v) for v in tr["succeeded_line_search"][0, 1:nq + 1]]
        replay_qp_counts(solver, x0[None], u0[None], N, 0.1, method, counts, succ)


def test_wide_model_refusals():
    from oracle import sqp as osqp
    from trajoptmpcreference_amd import TrajoptConstraint, _native
    n, N = 9, 8
    x0, u0 = osqp.initial_problem(_model(n), N, 0.1, 1)
    s = _solver(n)
    with pytest.raises(_native.NativeError, match="fp64 only"):
        s.SQP_batch(x0[None], u0[None], N, 0.1, "PCG-SS", {"precision": "fp32"})
    Nl = 60   # 60 x 18 = 1080 rows
    xl, ul = osqp.initial_problem(_model(n), Nl, 0.1, 2)
    with pytest.raises(_native.NativeError, match="N <= 56"):
        s.SQP_batch(xl[None], ul[None], Nl, 0.1, "PCG-SS", {})
    con = TrajoptConstraint(n, n, n, N)
    con.set_torque_limits([1.0] * n, [-1.0] * n, "AUGMENTED_LAGRANGIAN")
    with pytest.raises(_native.NativeError, match="box constraints with 9 joints"):
        _solver(n, con).SQP_batch(x0[None], u0[None], N, 0.1, "PCG-SS", {})


def test_wide_stream_equals_batch(ctx):
    """Continuous batching with a 9-joint chain (tmpc_sqp_solve_stream_device): every streamed problem's
    exit code, iterations and trajectories equal its batch solve's bitwise."""
    from oracle import sqp as osqp
    from trajoptmpcreference_amd import _native
    n, N = 9, 8
    m = _model(n)
    ctx.set_model(m)
    ctx.set_cost_quadratic(*quad_cost_arrays(n))
    base = _native.tmpc_options()
    ctx.lib.tmpc_default_options(base)
    ctx.options = base
    ctx.set_options()
    ctx.set_box_limits(None)
    xs, us = zip(*[osqp.initial_problem(m, N, 0.1, 950 + s) for s in range(6)])
    x, u = np.array(xs), np.array(us)
    ref = ctx.sqp_solve_batch(x, u, N, 0.1, "PCG-SS")
    s = ctx.solve_stream(x, u, N, 0.1, "PCG-SS", slots=4, copies=2)
    for p in range(12):
        i = p % 6
        assert int(s["exit"][p]) == int(ref["exit_sqp"][i]) and int(s["iters"][p]) == int(ref["sqp_iter"][i]), p
        assert np.array_equal(s["x"][p], ref["x"][i]) and np.array_equal(s["u"][p], ref["u"][i]), p


def test_wide_mpc_refused(ctx):
    from trajoptmpcreference_amd import _native
    n, N = 9, 8
    ctx.set_model(_model(n))
    ctx.set_cost_quadratic(*quad_cost_arrays(n))
    ctx.set_box_limits(None)
    with pytest.raises(_native.NativeError, match="MPC loop supports up to 7 joints"):
        ctx.mpc_batch(np.zeros((1, 2 * n, N)), np.zeros((1, n, N - 1)), N, 0.1, "PCG-SS", 2)


@pytest.mark.parametrize("n,N", [(9, 16), (12, 12)])
def test_wide_ilqr_matches_oracle(n, N):
    from oracle import ilqr as oilqr
    from oracle import sqp as osqp
    from test_gpu_ilqr import _check_full, _replay
    m = _model(n)
    solver = _solver(n)
    xs, us = zip(*[osqp.initial_problem(m, N, 0.1, 960 + i) for i in range(3)])
    r = solver.iLQR_batch(np.array(xs), np.array(us), N, 0.1, {})
    cost = osqp.QuadCost(*quad_cost_arrays(n))
    for i in range(3):
        with np.errstate(all="ignore"):
            _check_full(r, i, oilqr.ilqr(m, cost, xs[i], us[i], N, 0.1, {}))
    _replay(solver, r, m, cost, np.array(xs), np.array(us), N)
