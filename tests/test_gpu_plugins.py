"""GPU parity: the plugin-hook path (trajoptmpcreference_amd/hooks.py) against the REFERENCE's own runs
with the same user plugins (tests/golden/plugin_*.npz, written by make_golden.py run_plugins from
/root/reference/TrajoptMPCReference.py with the plugins of tests/plugin_models.py wrapped in its own
TrajoptCost / TrajoptPlant base classes):

  * CoupledCost -- a QuadraticCost subclass here that overrides value / gradient / hessian with a
    time-varying cost with an x-u cross term (its G_k is not block-diagonal) -- on arm3 N = 10;
  * SpringPlant -- a TrajoptPlant subclass without URDF (closed-form dynamics and gradient) with
    CoupledCost, N = 20;
  * CoupledCost with hard ACTIVE_SET torque limits on the 1-link arm (plugin_hard_*.npz, make_golden.py
    run_plugins_hard): the hooks' hard rows (TrajoptConstraint.py's value/jacobian at each knot) go through
    tmpc_qp_blocks_banded_batch -- the banded Schur path on the plugin's own blocks.

Integers exact against the reference's run: exit code, SQP iterations, line-search iterations, the
alpha path, the PCG count of every QP; J / c / merit / trajectories at 1e-7 relative.  Every QP is also
checked on identical inputs: the blocks the hooks formed are solved again with the Schur blocks returned
(tmpc_qp_blocks_batch), the count and dxul repeat bit for bit, and the canonical-order PCG
(oracle/canon.c) on that S takes the same count and returns the GPU's lambda bit for bit.  The direct
methods (N) against the reference's dense solve.  Pass-through subclasses of the built-ins (the F4
adapter) give the device path's answer."""
import glob
import os

import numpy as np
import pytest

import plugin_models as pm
from conftest import GOLDEN, quad_cost_arrays

pytestmark = pytest.mark.gpu

FILES = sorted(f for f in glob.glob(os.path.join(GOLDEN, "plugin_*.npz"))
               if not os.path.basename(f).startswith("plugin_hard_"))
HARD_FILES = sorted(glob.glob(os.path.join(GOLDEN, "plugin_hard_*.npz")))


def _classes():
    from trajoptmpcreference_amd import QuadraticCost, TrajoptCost, TrajoptPlant

    class CoupledQuadratic(QuadraticCost):
        """a QuadraticCost whose hooks the caller replaced"""

        def __init__(self, nx, nu):
            Q, QF, R, M, xg, w = pm.coupled_arrays(nx, nu)
            super().__init__(Q, QF, R, xg)
            self.arrs = (Q, QF, R, M, xg, w)

        def value(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_value(x, u, timestep, self.arrs)

        def gradient(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_gradient(x, u, timestep, self.arrs)

        def hessian(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_hessian(x, u, timestep, self.arrs)

    class CoupledCost(TrajoptCost):
        def __init__(self, nx, nu):
            self.arrs = pm.coupled_arrays(nx, nu)

        def value(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_value(x, u, timestep, self.arrs)

        def gradient(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_gradient(x, u, timestep, self.arrs)

        def hessian(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_hessian(x, u, timestep, self.arrs)

    class SpringPlant(TrajoptPlant):
        def forward_dynamics(self, x, u, *a, **k):
            return pm.spring_qdd(np.asarray(x, dtype=float), np.asarray(u, dtype=float))

        def forward_dynamics_gradient(self, x, u, *a, **k):
            return pm.spring_dqdd(np.asarray(x, dtype=float), np.asarray(u, dtype=float))

        def get_num_pos(self):
            return pm.NQ

        def get_num_vel(self):
            return pm.NQ

        def get_num_cntrl(self):
            return pm.NQ

    return CoupledQuadratic, CoupledCost, SpringPlant


def _solver(which):
    from trajoptmpcreference_amd import TrajoptMPCReference, URDFPlant, planar_arm_urdf
    CoupledQuadratic, CoupledCost, SpringPlant = _classes()
    if which == "cost":
        return TrajoptMPCReference(URDFPlant(options={"path_to_urdf": planar_arm_urdf(3)}), CoupledQuadratic(6, 3))
    return TrajoptMPCReference(SpringPlant(), CoupledCost(4, 2))


@pytest.mark.parametrize("f", FILES, ids=lambda f: os.path.basename(f))
def test_plugin_sqp_matches_reference(f, monkeypatch):
    from oracle import canon
    from trajoptmpcreference_amd import _native
    which, Ns, _, method = os.path.basename(f)[7:-4].split("_")
    N = int(Ns[1:])
    d = np.load(f)
    solver = _solver(which)
    calls = []
    orig = _native.Context.qp_blocks_batch

    def spy(self, *a, **k):
        r = orig(self, *a, **k)
        calls.append((a, k, r))
        return r

    monkeypatch.setattr(_native.Context, "qp_blocks_batch", spy)
    x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(d["x0"], d["u0"], N, float(d["dt"]), method, {})
    monkeypatch.setattr(_native.Context, "qp_blocks_batch", orig)
    assert (exit_sqp, sqp_iter, exit_soft, outer_iter) == (int(d["exit_sqp"]), int(d["sqp_iter"]),
                                                           int(d["exit_soft"]), int(d["outer_iter"]))
    tr = solver.trace
    assert [t["alpha"] for t in tr] == list(d["tr_alpha"])
    assert [t["line_search_iteration"] for t in tr] == list(d["tr_line_search_iteration"].astype(int))
    assert [t["succeeded_line_search"] for t in tr] == list(d["tr_succeeded_line_search"].astype(bool))
    if method.startswith("PCG"):
        assert [t["inner_iters"] for t in tr[1:]] == list(d["pcg_iters"])
    for key in ("J", "c", "merit", "rho"):
        assert np.allclose([t[key] for t in tr], d["tr_" + key], rtol=1e-7, atol=1e-12), key
    scale = max(1.0, float(np.max(np.abs(d["x"]))))
    assert float(np.max(np.abs(x - d["x"]))) < 1e-7 * scale
    scale = max(1.0, float(np.max(np.abs(d["u"]))))
    assert float(np.max(np.abs(u - d["u"]))) < 1e-7 * scale
    # every QP on identical inputs: the same blocks again (with S out) and the canonical-order PCG
    assert len(calls) == len(tr) - 1
    ctx = _native.default_context(0)
    nx = 2 * solver.plant.get_num_cntrl()
    for j, (a, k, r) in enumerate(calls):
        G, g, A, Bm, c, rho, meth = a
        assert np.allclose(r["dxul"][0], d["dxul"][j], rtol=1e-6, atol=1e-9 * max(1.0, np.abs(d["dxul"][j]).max()))
        if not meth.startswith("PCG"):
            continue
        q = ctx.qp_blocks_batch(G, g, A, Bm, c, rho, meth, want_blocks=True)
        assert int(q["pcg_iters"][0]) == int(r["pcg_iters"][0])
        assert np.array_equal(q["dxul"], r["dxul"]), j
        lam, it, _ = canon.pcg(q["S_diag"][0], q["S_lo"][0], q["gamma"][0], meth[4:])
        assert it == int(r["pcg_iters"][0]), (j, it, int(r["pcg_iters"][0]))
        assert np.array_equal(lam, r["dxul"][0][-N * nx:]), j


def test_pass_through_subclasses_match_the_device_path():
    """The F4 adapter pattern (a QuadraticCost subclass whose hooks forward to QuadraticCost's) and a
    URDFPlant subclass forwarding its dynamics take the plugin-hook path and land on the device path's
    answer: integers identical, trajectories within 1e-9."""
    from oracle import sqp as osqp
    from conftest import arm_model
    from trajoptmpcreference_amd import QuadraticCost, TrajoptMPCReference, URDFPlant, planar_arm_urdf

    class PassCost(QuadraticCost):
        def value(self, x, u=None, timestep=None, *a, **k):
            return QuadraticCost.value(self, x, u, timestep)

        def gradient(self, x, u=None, timestep=None, *a, **k):
            return QuadraticCost.gradient(self, x, u, timestep)

        def hessian(self, x, u=None, timestep=None, *a, **k):
            return QuadraticCost.hessian(self, x, u, timestep)

    class PassPlant(URDFPlant):
        def integrator(self, xk, uk, dt, return_gradient=False, *a, **k):
            return URDFPlant.integrator(self, xk, uk, dt, return_gradient)

    path = planar_arm_urdf(3)
    x0, u0 = osqp.initial_problem(arm_model("arm3"), 12, 0.1, 31)
    ref = TrajoptMPCReference(URDFPlant(options={"path_to_urdf": path}), QuadraticCost(*quad_cost_arrays(3)))
    r0 = ref.SQP(x0, u0, 12, 0.1, "PCG-SS", {})
    for plant, cost in ((URDFPlant(options={"path_to_urdf": path}), PassCost(*quad_cost_arrays(3))),
                        (PassPlant(options={"path_to_urdf": path}), QuadraticCost(*quad_cost_arrays(3)))):
        s = TrajoptMPCReference(plant, cost)
        assert s._hooks()
        r = s.SQP(x0, u0, 12, 0.1, "PCG-SS", {})
        assert (r[2], r[5]) == (r0[2], r0[5])
        assert [t["alpha"] for t in s.trace] == [t["alpha"] for t in ref.trace]
        assert [t["inner_iters"] for t in s.trace] == [t["inner_iters"] for t in ref.trace]
        assert np.allclose(r[0], r0[0], rtol=1e-9, atol=1e-12)
        assert np.allclose(r[1], r0[1], rtol=1e-9, atol=1e-12)


def test_plugin_qp_level_methods():
    """solveKKTSystem_Schur / solveKKTSystem with user plugins: the hooks form the blocks, the GPU solves;
    against the dense KKT system built from formKKTSystemBlocks (the same hooks): residual at rounding."""
    solver = _solver("plant")
    N, dt = 12, 0.1
    x, u = pm.spring_initial(N, dt, 5)
    xs = x[:, 0].copy()
    G, g, C, c = solver.formKKTSystemBlocks(x, u, xs, N, dt)
    rho = 1e-3
    K = np.block([[G + rho * np.eye(G.shape[0]), C.T], [C, np.zeros((C.shape[0], C.shape[0]))]])
    rhs = np.vstack((g, c))
    for dxul in (solver.solveKKTSystem(x, u, xs, N, dt, rho),
                 solver.solveKKTSystem_Schur(x, u, xs, N, dt, rho, use_PCG=True,
                                             options={"preconditioner_type": "SS", "exit_tolerance": 1e-12,
                                                      "max_iter": 500})):
        res = float(np.max(np.abs(K @ dxul - rhs)))
        assert res < 1e-8 * max(1.0, float(np.max(np.abs(rhs)))), res


def test_plugin_qp_with_an_indefinite_hessian_block():
    """(G_k + rho I)^-1 of the plugin-hook QP by Gauss-Jordan with partial pivoting: knot blocks
    that are indefinite and whose leading entry cancels rho exactly (a zero first pivot -- LinAlgError for an
    unpivoted elimination, invertible for np.linalg.inv) give the dense KKT solution of
    solveKKTSystem (:313-359), methods N and S."""
    from trajoptmpcreference_amd import _native
    rng = np.random.default_rng(11)
    nu, N, rho = 3, 6, 1e-3
    nx, n = 2 * nu, 3 * nu
    G = np.zeros((1, N, n, n))
    for k in range(N):
        m = n if k < N - 1 else nx
        M = rng.uniform(-1.0, 1.0, (m, m))
        H = M + M.T + np.diag(rng.choice([-3.0, 3.0], m))   # indefinite, well conditioned
        H[0, 0] = -rho                                        # first pivot of H + rho I exactly zero
        G[0, k, :m, :m] = H
    g = rng.uniform(-1.0, 1.0, (1, N, n))
    A = rng.uniform(-0.3, 0.3, (1, N - 1, nx, nx)) + np.eye(nx)
    Bm = rng.uniform(-0.3, 0.3, (1, N - 1, nx, nu))
    c = rng.uniform(-0.1, 0.1, (1, N, nx))
    # the dense KKT system of formKKTSystemBlocks' blocks (:200-271) with rho on G's diagonal (:319-322)
    nz = n * (N - 1) + nx
    Gd = np.zeros((nz, nz))
    gd = np.zeros(nz)
    C = np.zeros((nx * N, nz))
    cd = c[0].reshape(-1)
    C[:nx, :nx] = np.eye(nx)
    for k in range(N):
        m = n if k < N - 1 else nx
        Gd[k * n:k * n + m, k * n:k * n + m] = G[0, k, :m, :m]
        gd[k * n:k * n + m] = g[0, k, :m]
        if k < N - 1:
            C[(k + 1) * nx:(k + 2) * nx, k * n:k * n + nx] = -A[0, k]
            C[(k + 1) * nx:(k + 2) * nx, k * n + nx:k * n + n] = -Bm[0, k]
            C[(k + 1) * nx:(k + 2) * nx, (k + 1) * n:(k + 1) * n + nx] = np.eye(nx)
    K = np.block([[Gd + rho * np.eye(nz), C.T], [C, np.zeros((nx * N, nx * N))]])
    ref = np.linalg.solve(K, np.concatenate([gd, cd]))
    ctx = _native.default_context(0)
    for meth, tol in (("N", 1e-9), ("S", 1e-9)):
        r = ctx.qp_blocks_batch(G, g, A, Bm, c, rho, meth, want_blocks=False)
        got = r["dxul"][0]
        assert np.all(np.isfinite(got)), meth
        assert np.max(np.abs(got[:nz] - ref[:nz])) < tol * max(1.0, np.max(np.abs(ref[:nz]))), meth


@pytest.mark.parametrize("f", HARD_FILES, ids=lambda f: os.path.basename(f))
def test_plugin_cost_with_hard_limits_matches_reference(f, monkeypatch):
    """A user cost plugin AND hard ACTIVE_SET torque limits (TrajoptMPCReference.py:238-248 appends the
    constraint's rows to C after each knot's dynamics rows, on the plugin's own blocks) against the
    reference's own run: exit code, SQP iterations, every QP's active set (bit 4 = a row of sign +1 active at
    the knot, bit 5 = sign -1, read back from the reference's own C), the alpha path, line-search iterations,
    every PCG count exact; J / c / merit / trajectories at 1e-7.  Every PCG QP is replayed on its own S:
    the canonical-order PCG (oracle/hard.py) takes the GPU's count."""
    from oracle import hard as ohard
    from trajoptmpcreference_amd import TrajoptConstraint, TrajoptMPCReference, URDFPlant, _native
    _, CoupledCost, _ = _classes()
    d = np.load(f)
    N = d["x0"].shape[1]
    method = os.path.basename(f)[:-4].split("_")[-1]
    con = TrajoptConstraint(1, 1, 1, N)
    con.set_torque_limits([float(d["ub"])], [float(d["lb"])], "ACTIVE_SET")
    solver = TrajoptMPCReference(URDFPlant(options={"path_to_urdf": str(d["urdf"])}), CoupledCost(2, 1), con)
    assert solver._hooks()
    calls = []
    orig = _native.Context.qp_blocks_banded_batch

    def spy(self, G, *a, **k):
        r = orig(self, G, *a, **k)
        calls.append((r, self.qp_hard_info(G.shape[0], G.shape[1]) if method.startswith("PCG") else None))
        return r

    monkeypatch.setattr(_native.Context, "qp_blocks_banded_batch", spy)
    x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(d["x0"], d["u0"], N, float(d["dt"]), method, {})
    monkeypatch.setattr(_native.Context, "qp_blocks_banded_batch", orig)
    assert (exit_sqp, sqp_iter, exit_soft, outer_iter) == (int(d["exit_sqp"]), int(d["sqp_iter"]),
                                                           int(d["exit_soft"]), int(d["outer_iter"]))
    ref_masks = [[0] * N for _ in range(len(d["C_rows"]))]
    for q, k, sg in zip(d["act_qp"], d["act_knot"], d["act_sign"]):
        ref_masks[int(q)][int(k)] |= 1 << (4 if int(sg) > 0 else 5)
    assert solver.active_sets == ref_masks
    assert max(max(m) for m in ref_masks) > 0   # the limits bind
    tr = solver.trace
    assert [t["alpha"] for t in tr] == list(d["tr_alpha"])
    assert [t["line_search_iteration"] for t in tr] == list(d["tr_line_search_iteration"].astype(int))
    assert [t["succeeded_line_search"] for t in tr] == list(d["tr_succeeded_line_search"].astype(bool))
    if method.startswith("PCG"):
        assert [t["inner_iters"] for t in tr[1:]] == list(d["pcg_iters"])
    for key in ("J", "c", "merit"):
        assert np.allclose([t[key] for t in tr], d["tr_" + key], rtol=1e-7, atol=1e-12), key
    assert np.allclose(x, d["x"], rtol=1e-7, atol=1e-10)
    assert np.allclose(u, d["u"], rtol=1e-7, atol=1e-10)
    assert len(calls) == len(tr) - 1
    if not method.startswith("PCG"):
        return
    opts = {}
    solver.set_default_options(opts)
    for j, (r, info) in enumerate(calls):
        D = int(info["dim"][0])
        assert D >= N * 2
        S = _unband_S(info["S_band"][0], info["W"], D)
        _, it = ohard.pcg_canonical(S, info["gamma"][0, :D], 2, method[4:], opts["exit_tolerance_linSys"],
                                    opts["max_iter_linSys"])
        assert it == int(r["pcg_iters"][0]), (j, it, int(r["pcg_iters"][0]))


def _unband_S(Sb, W, D):
    S = np.zeros((D, D))
    for o in range(2 * W + 1):
        a = np.arange(D)
        c = a - W + o
        ok = (c >= 0) & (c < D)
        S[a[ok], c[ok]] = Sb[a[ok], o]
    return S


@pytest.mark.parametrize("method", ["S", "N", "PCG-SS", "PCG-BJ"])
def test_plugin_qp_past_1024_rows(method):
    """The plugin-hook QP past the 1024-row dense kernels (N * nx = 1200: arm6-sized blocks, N = 100) goes
    through tmpc_qp_blocks_banded_batch with no hard rows: the direct methods give the dense KKT solution of
    the same blocks (solveKKTSystem, TrajoptMPCReference.py:313-359); the PCG's count is the canonical-order
    PCG's on the QP's own S and its lambda solves S lambda = gamma to the PCG's tolerance."""
    from oracle import hard as ohard
    from trajoptmpcreference_amd import _native
    rng = np.random.default_rng(21)
    nu, N, rho = 6, 100, 1e-3
    nx, n = 2 * nu, 3 * nu
    G = np.zeros((1, N, n, n))
    for k in range(N):
        m = n if k < N - 1 else nx
        M = rng.uniform(-1.0, 1.0, (m, m))
        G[0, k, :m, :m] = M @ M.T / m + np.eye(m)
    g = rng.uniform(-1.0, 1.0, (1, N, n))
    A = rng.uniform(-0.05, 0.05, (1, N - 1, nx, nx)) + np.eye(nx)
    A[0, :, :nu, nu:] += 0.1 * np.eye(nu)
    Bm = rng.uniform(-0.1, 0.1, (1, N - 1, nx, nu))
    c = rng.uniform(-0.1, 0.1, (1, N, nx))
    nz = n * (N - 1) + nx
    Gd = np.zeros((nz, nz))
    gd = np.zeros(nz)
    C = np.zeros((nx * N, nz))
    C[:nx, :nx] = np.eye(nx)
    for k in range(N):
        m = n if k < N - 1 else nx
        Gd[k * n:k * n + m, k * n:k * n + m] = G[0, k, :m, :m]
        gd[k * n:k * n + m] = g[0, k, :m]
        if k < N - 1:
            C[(k + 1) * nx:(k + 2) * nx, k * n:k * n + nx] = -A[0, k]
            C[(k + 1) * nx:(k + 2) * nx, k * n + nx:k * n + n] = -Bm[0, k]
            C[(k + 1) * nx:(k + 2) * nx, (k + 1) * n:(k + 1) * n + nx] = np.eye(nx)
    K = np.block([[Gd + rho * np.eye(nz), C.T], [C, np.zeros((nx * N, nx * N))]])
    ref = np.linalg.solve(K, np.concatenate([gd, c[0].reshape(-1)]))
    ctx = _native.default_context(0)
    rows = [[[] for _ in range(N)]]
    r = ctx.qp_blocks_banded_batch(G, g, A, Bm, c, rho, rows, method)
    got = r["dxul"][0]
    assert got.shape == ref.shape and np.all(np.isfinite(got))
    if not method.startswith("PCG"):
        assert np.max(np.abs(got - ref)) < 1e-8 * max(1.0, np.max(np.abs(ref))), method
        return
    info = ctx.qp_hard_info(1, N)
    D = int(info["dim"][0])
    assert D == N * nx
    S = _unband_S(info["S_band"][0], info["W"], D)
    gam = info["gamma"][0, :D]
    tol, max_iter = ctx.options.exit_tolerance_linSys, ctx.options.max_iter_linSys
    lam_c, it = ohard.pcg_canonical(S, gam, nx, method[4:], tol, max_iter)
    assert it == int(r["pcg_iters"][0]), (it, int(r["pcg_iters"][0]))
    lam = got[nz:]
    assert np.max(np.abs(lam - lam_c)) < 1e-9 * max(1.0, np.max(np.abs(lam_c)))
    # the primal step from lambda: within the PCG's tolerance of the exact KKT solution
    assert np.max(np.abs(got[:nz] - ref[:nz])) < 1e-3 * max(1.0, np.max(np.abs(ref[:nz])))
