"""Continuous batching (tmpc_sqp_solve_stream_device / tmpc_ilqr_solve_stream_device, ABI 10).

A stream of P problems runs through B < P resident slots: a slot whose problem finishes takes the next
pending one in the same batch iteration, so most problems ENTER MID-STREAM, next to problems that are
half-way through their solve.  Each problem's operations are those of a batch solve from the same input,
so every output must equal the batch solve's bit for bit: trajectories, exit codes, iteration counts,
outer passes and every used trace row (PCG counts, alpha path, J, c, merit, rho ...).  The batch solves
themselves are pinned to the reference / oracle by the other GPU tests (test_gpu_sqp, _soft, _hard,
_ilqr, _configs); this file extends test_batch_equals_single to problems that enter mid-stream.
Problems are solved `copies` times (stream problem p = input p % P0): later copies enter slots in other
states and must still reproduce copy 0 bitwise."""
import numpy as np
import pytest

from conftest import arm_model, quad_cost_arrays

pytestmark = pytest.mark.gpu


def _setup(ctx, n, limits=None, **opts):
    from trajoptmpcreference_amd import _native
    ctx.set_model(arm_model({2: "arm2", 3: "arm3", 6: "arm6fix"}[n]))
    ctx.set_cost_quadratic(*quad_cost_arrays(n))
    base = _native.tmpc_options()
    ctx.lib.tmpc_default_options(base)
    ctx.options = base
    ctx.set_options(**opts)
    ctx.set_box_limits(limits)


def _problems(n, N, seeds, dt=0.1, scale=1.0):
    from oracle import sqp as osqp
    m = arm_model({2: "arm2", 3: "arm3", 6: "arm6fix"}[n])
    xs, us = zip(*[osqp.initial_problem(m, N, dt, int(s)) for s in seeds])
    x, u = np.array(xs), np.array(us)
    x[:, : n, 0] *= scale
    return x, u


def _batch(ctx, solver, x, u, N, dt, soft):
    if soft:
        ctx.set_soft_state(x.shape[0], N)   # the batch starts from the initial constants, as each stream problem
    if solver == "iLQR":
        r = ctx.ilqr_solve_batch(x, u, N, dt)
        return dict(x=r["x"], u=r["u"], exit=r["exit_code"], iters=r["iter"], exit_soft=r["exit_soft"],
                    outer_iter=r["outer_iter"], trace=r["trace"])
    r = ctx.sqp_solve_batch(x, u, N, dt, solver)
    return dict(x=r["x"], u=r["u"], exit=r["exit_sqp"], iters=r["sqp_iter"], exit_soft=r["exit_soft"],
                outer_iter=r["outer_iter"], trace=r["trace"])


def _assert_stream_equals_batch(ctx, solver, x, u, N, slots, copies, dt=0.1, soft=False, substreams=1):
    ref = _batch(ctx, solver, x, u, N, dt, soft)
    s = ctx.solve_stream(x, u, N, dt, solver, slots=slots, copies=copies, substreams=substreams)
    P0 = x.shape[0]
    for p in range(P0 * copies):
        i = p % P0
        for k in ("exit", "iters", "exit_soft", "outer_iter"):
            assert int(s[k][p]) == int(ref[k][i]), (p, k, int(s[k][p]), int(ref[k][i]))
        assert np.array_equal(s["x"][p], ref["x"][i]), p
        assert np.array_equal(s["u"][p], ref["u"][i]), p
        rows = int(ref["iters"][i]) + (1 if int(ref["exit"][i]) == 3 else 0) + 1   # row 0 + one per QP
        for name, a in ref["trace"].items():
            assert np.array_equal(s["trace"][name][p, :rows], a[i, :rows], equal_nan=True), (p, name)
    return ref, s


def test_stream_sqp_pcg_ss_arm3_equals_batch(ctx):
    _setup(ctx, 3)
    x, u = _problems(3, 16, range(24))
    ref, s = _assert_stream_equals_batch(ctx, "PCG-SS", x, u, 16, slots=5, copies=3)
    assert len(set(int(v) for v in ref["iters"])) > 1   # problems finish at different iterations


def test_stream_sqp_headline_arm6_n64_equals_batch(ctx):
    """the headline workload (arm6 N = 64, PCG-SS): 12 problems x 2 copies through 7 slots"""
    _setup(ctx, 6)
    x, u = _problems(6, 64, range(12))
    _assert_stream_equals_batch(ctx, "PCG-SS", x, u, 64, slots=7, copies=2)


@pytest.mark.parametrize("method", ["S", "PCG-J", "PCG-BJ"])
def test_stream_sqp_methods_equal_batch(ctx, method):
    _setup(ctx, 3)
    x, u = _problems(3, 12, range(100, 110))
    _assert_stream_equals_batch(ctx, method, x, u, 12, slots=3, copies=2)


def test_stream_sqp_soft_limits_equal_batch(ctx):
    """augmented-Lagrangian torque + joint limits (config 4's kind): outer passes restart per problem inside
    the stream; every stream problem starts from the initial constants"""
    lim = {"torque": dict(mode="AUGMENTED_LAGRANGIAN", lb=-0.5, ub=0.5),
           "joint": dict(mode="AUGMENTED_LAGRANGIAN", lb=-1.0, ub=1.0)}
    _setup(ctx, 3, lim)
    x, u = _problems(3, 16, range(200, 212))
    ref, _ = _assert_stream_equals_batch(ctx, "PCG-SS", x, u, 16, slots=4, copies=2, soft=True)
    assert max(int(v) for v in ref["outer_iter"]) > 1


def test_stream_sqp_hard_limits_equal_batch(ctx):
    """ACTIVE_SET torque + velocity rows (the banded Schur path)"""
    lim = {"torque": dict(mode="ACTIVE_SET", lb=-0.5, ub=0.5), "velocity": dict(mode="ACTIVE_SET", lb=-1.0, ub=1.0)}
    _setup(ctx, 3, lim)
    x, u = _problems(3, 16, range(300, 310))
    _assert_stream_equals_batch(ctx, "PCG-SS", x, u, 16, slots=3, copies=2)


def test_stream_sqp_pcg_warm_start_equals_batch(ctx):
    """each QP's PCG starts from the problem's previous lambda: a refilled slot starts from zeros again"""
    _setup(ctx, 3, pcg_warm_start=1)
    x, u = _problems(3, 16, range(400, 410))
    _assert_stream_equals_batch(ctx, "PCG-SS", x, u, 16, slots=3, copies=2)


def test_stream_ilqr_equals_batch(ctx):
    _setup(ctx, 3)
    x, u = _problems(3, 16, range(500, 516))
    ref, _ = _assert_stream_equals_batch(ctx, "iLQR", x, u, 16, slots=5, copies=2)
    assert len(set(int(v) for v in ref["iters"])) > 1


def test_stream_ilqr_augmented_lagrangian_equals_batch(ctx):
    """config 3's kind (iLQR + AL torque limits)"""
    _setup(ctx, 3, {"torque": dict(mode="AUGMENTED_LAGRANGIAN", lb=-0.5, ub=0.5)})
    x, u = _problems(3, 16, range(600, 610))
    _assert_stream_equals_batch(ctx, "iLQR", x, u, 16, slots=3, copies=2, soft=True)


def test_stream_more_slots_than_problems(ctx):
    """slots > problems: every problem gets its own slot, nothing pending"""
    _setup(ctx, 2)
    x, u = _problems(2, 10, range(3))
    _assert_stream_equals_batch(ctx, "PCG-SS", x, u, 10, slots=8, copies=1)


def test_stream_counts_every_problem_once(ctx):
    """the stream's work counters are the sum of the batch solves' (each problem's QPs counted once)"""
    _setup(ctx, 3)
    x, u = _problems(3, 12, range(700, 709))
    ctx.sqp_solve_batch(x, u, 12, 0.1, "PCG-SS", with_trace=False)
    cb = ctx.solve_counters()
    ctx.solve_stream(x, u, 12, 0.1, "PCG-SS", slots=2, copies=2, with_trace=False)
    cs = ctx.solve_counters()
    assert cs[0] == 2 * cb[0] and cs[1] == 2 * cb[1] and cs[2] == 2 * cb[2], (cs, cb)


@pytest.mark.parametrize("solver,K", [("PCG-SS", 2), ("PCG-SS", 3), ("iLQR", 2)])
def test_stream_substreams_equal_batch(ctx, solver, K):
    """K concurrent sub-streams (own HIP stream, slots / K slots, a contiguous 1 / K of the problems each, host
    threads): every problem's results still equal its batch solve's bitwise, at its global output row"""
    _setup(ctx, 3, {"torque": dict(mode="AUGMENTED_LAGRANGIAN", lb=-0.5, ub=0.5)})
    x, u = _problems(3, 16, range(800, 811))
    _assert_stream_equals_batch(ctx, solver, x, u, 16, slots=6, copies=2, soft=True, substreams=K)


def test_stream_substreams_count_every_problem_once(ctx):
    _setup(ctx, 3)
    x, u = _problems(3, 12, range(900, 907))
    ctx.sqp_solve_batch(x, u, 12, 0.1, "PCG-SS", with_trace=False)
    cb = ctx.solve_counters()
    ctx.solve_stream(x, u, 12, 0.1, "PCG-SS", slots=4, copies=3, with_trace=False, substreams=2)
    cs = ctx.solve_counters()
    assert cs[:3] == [3 * v for v in cb[:3]], (cs, cb)
