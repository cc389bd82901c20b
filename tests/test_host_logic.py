"""CPU: host-side logic of the drop-in classes -- argument validation, option
defaults, cost plugin arithmetic, block extraction -- and the guarantee that
the product path has no CPU fallback (without a GPU it raises instead of
computing)."""
import numpy as np
import pytest

from conftest import arm_model, quad_cost_arrays


def _solver(n=3):
    from trajoptmpcreference_amd import QuadraticCost, TrajoptMPCReference, URDFPlant, planar_arm_urdf
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
    return TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(n)))


def test_plugin_type_checks_raise_instead_of_exit():
    """TrajoptMPCReference.py:32-39 print+exit() on wrong plugin types; here TypeError."""
    from trajoptmpcreference_amd import QuadraticCost, TrajoptMPCReference, URDFPlant, planar_arm_urdf
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(2)})
    cost = QuadraticCost(*quad_cost_arrays(2))
    with pytest.raises(TypeError):
        TrajoptMPCReference("plant", cost)
    with pytest.raises(TypeError):
        TrajoptMPCReference(plant, object())
    with pytest.raises(TypeError):
        TrajoptMPCReference(plant, cost, constraintObj=3)
    s = TrajoptMPCReference(plant, cost)
    with pytest.raises(TypeError):
        s.update_cost(None)
    with pytest.raises(TypeError):
        s.update_plant(None)


def test_solver_default_options_mutate_the_callers_dict():
    """set_default_options (:91-115) fills the caller's dict in place."""
    s = _solver()
    o = {"max_iter_SQP_DDP": 7}
    s.set_default_options(o)
    assert o["max_iter_SQP_DDP"] == 7
    assert o["exit_tolerance_linSys"] == 1e-6 and o["max_iter_linSys"] == 100
    assert o["rho_init_SQP_DDP"] == 0.001 and o["rho_max_SQP_DDP"] == 1e3
    assert o["expected_reduction_min_SQP_DDP"] == 0.05 and o["expected_reduction_max_SQP_DDP"] == 3
    assert o["overloading"] is False


def test_invalid_method_and_unsupported_paths_raise():
    s = _solver()
    x = np.zeros((6, 8))
    u = np.zeros((3, 7))
    with pytest.raises(ValueError):
        s.SQP(x, u, 8, 0.1, "CG", {})
    with pytest.raises(NotImplementedError):
        s.SQP(x, u, 8, 0.1, "PCG-SS", {"overloading": True})


def test_plant_validation():
    from trajoptmpcreference_amd import URDFPlant, planar_arm_urdf
    from trajoptmpcreference_amd.plant import TrajoptPlant
    with pytest.raises(ValueError):
        TrajoptPlant(integrator_type=9)
    with pytest.raises(NotImplementedError):
        TrajoptPlant(integrator_type=4)
    with pytest.raises(ValueError):
        TrajoptPlant(need_path=True)
    p = URDFPlant(options={"path_to_urdf": planar_arm_urdf(6)})
    assert (p.get_num_pos(), p.get_num_vel(), p.get_num_cntrl()) == (6, 6, 6)
    assert p.rbdReference.overloading is False


def test_quadratic_cost_matches_oracle_and_accepts_iter_kwargs():
    """QuadraticCost value/gradient/hessian (TrajoptCost.py:24-104), including the
    iter_* tracing kwargs the reference's own class rejects."""
    from oracle.sqp import QuadCost
    from trajoptmpcreference_amd import QuadraticCost
    rng = np.random.default_rng(3)
    Q, QF, R, xg = quad_cost_arrays(3)
    xg = rng.normal(size=6)
    c = QuadraticCost(Q, QF, R, xg, QF_start=5)
    o = QuadCost(Q, QF, R, xg, QF_start=5)
    x, u = rng.normal(size=6), rng.normal(size=3)
    for k in (0, 4, 5, 9):
        assert np.isclose(c.value(x, u, k, iter_1=1, iter_2=2, iter_3=3), o.value(x, u, k))
        assert np.allclose(np.ravel(c.gradient(x, u, k, iter_1=1)), np.ravel(o.gradient(x, u, k)))
        assert np.allclose(c.hessian(x, u, k), o.hessian(False, k))
    assert np.isclose(c.value(x), o.value(x, None, 0))
    assert np.allclose(c.hessian(x), o.hessian(True, 0))


def test_pcg_block_extraction():
    """The PCG class accepts only block-tridiagonal A (the Schur complement's structure)."""
    from oracle.sqp import dense_from_blocks
    from trajoptmpcreference_amd.pcg import PCG, extract_blocks
    rng = np.random.default_rng(0)
    Dg, Lo = rng.normal(size=(4, 3, 3)), rng.normal(size=(3, 3, 3))
    Up = np.transpose(Lo, (0, 2, 1))
    A = dense_from_blocks(Dg, Lo, Up)
    d, l, up = extract_blocks(A, 3)
    assert np.array_equal(d, Dg) and np.array_equal(l, Lo) and np.array_equal(up, Up)
    A[0, 11] = 1.0
    with pytest.raises(ValueError):
        extract_blocks(A, 3)
    with pytest.raises(ValueError):
        extract_blocks(np.zeros((10, 10)), 3)
    with pytest.raises(ValueError):
        PCG(A, np.zeros(12), 3, 4, options={"preconditioner_type": "XX"})
    p = PCG(dense_from_blocks(Dg, Lo, Up), np.zeros(12), 3, 4)
    assert p.options["preconditioner_type"] == "BJ" and p.options["exit_tolerance"] == 1e-6


def test_urdf_generator_round_trip_and_tree_detection():
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    m = parse_urdf(planar_arm_urdf(4))
    assert m.n == 4 and list(m.parent) == [-1, 0, 1, 2] and m.is_serial_chain()
    assert np.allclose(m.X(0, 0.0), m.X0[0] + m.Xa[0])


def test_no_cpu_fallback_without_gpu():
    """On a host without a GPU the solver raises -- it never computes on the CPU."""
    from trajoptmpcreference_amd import _native
    if _native.device_count() > 0:
        pytest.skip("a GPU is present")
    s = _solver(2)
    from oracle.sqp import initial_problem
    x, u = initial_problem(arm_model("arm2"), 8, 0.1, 0)
    with pytest.raises(_native.NativeError):
        s.SQP(x, u, 8, 0.1, "PCG-SS", {})


def test_bench_cpu_baseline_runs_the_oracle_on_a_bounded_sample():
    """bench.py's cpu_baseline leg: the oracle restatement of the same workload; it also returns the
    per-problem integers the bench's parity check compares with the GPU."""
    import bench
    v, wall, res = bench.cpu_baseline(2, 8, 2, 2, 0)
    assert v > 0 and wall > 0 and len(res) == 2
    assert all(r["exit_sqp"] in (1, 2, 3) and len(r["pcg_iters"]) >= r["sqp_iter"] for r in res)
    # parity_check against itself dressed as a GPU result: zero mismatches
    B, W = len(res), 101
    gpu = {"exit_sqp": np.array([r["exit_sqp"] for r in res]), "sqp_iter": np.array([r["sqp_iter"] for r in res]),
           "x": np.array([r["x"] for r in res]), "u": np.array([r["u"] for r in res]),
           "trace": {"pcg_iters": np.zeros((B, W), dtype=np.int32)}}
    for i, r in enumerate(res):
        gpu["trace"]["pcg_iters"][i, 1:1 + len(r["pcg_iters"])] = r["pcg_iters"]
    p = bench.parity_check(gpu, res)
    assert p["checked"] == 2 and p["mismatches"] == 0 and p["max_traj_rel_diff"] == 0.0
    gpu["trace"]["pcg_iters"][1, 1] += 1
    assert bench.parity_check(gpu, res)["mismatches"] == 1


def test_bench_hard_line_oracle_solve():
    """bench.py's hard-limit line checks the GPU against the oracle's solve under the same preset
    (ACTIVE_SET torque + velocity rows, canonical-order PCG): a small instance runs and returns the
    integers parity_check compares."""
    import bench
    r = bench._cpu_solve_hard((0, 2, 8))
    assert r["exit_sqp"] in (1, 2, 3, 4) and len(r["pcg_iters"]) >= r["sqp_iter"]
    assert r["x"].shape == (4, 8) and r["u"].shape == (2, 7)


def test_bench_byte_and_flop_models():
    """b_pcg = 8 (2 (2N-1) nx^2 + 10 N nx) = 354,048 B/iteration and
    f_pcg = 2*3*nx^2*N*2 + 10*N*nx = 118,272 flop/iteration for arm6 N=64."""
    import bench
    assert bench.b_pcg_survey(64, 12) == 354048
    assert bench.f_pcg_survey(64, 12) == 118272
    assert bench.pcg_flops_impl(64, 12, "PCG-SS") > bench.pcg_flops_impl(64, 12, "PCG-BJ")


def test_pendulum_model_closed_form():
    """PendulumPlant's model (urdf.pendulum_urdf): the oracle's dynamics equal
    qdd = (u - m g l sin q) / (m l^2 + I_bob) (the plant examples/pendulum.py needs)."""
    from oracle import rbd
    from trajoptmpcreference_amd.urdf import parse_urdf, pendulum_urdf
    m = parse_urdf(pendulum_urdf(mass=2.0, length=0.5))
    rng = np.random.default_rng(0)
    x = np.column_stack([rng.uniform(-3, 3, 8), rng.uniform(-2, 2, 8)])
    u = rng.uniform(-5, 5, (8, 1))
    qdd = (rbd.euler(m, x, u, 1.0)[:, 1] - x[:, 1])
    ref = (u[:, 0] - 2.0 * 9.81 * 0.5 * np.sin(x[:, 0])) / (2.0 * 0.25 + 1e-3)
    assert np.allclose(qdd, ref, rtol=1e-12, atol=1e-12)
