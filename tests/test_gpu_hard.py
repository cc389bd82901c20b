"""GPU parity: hard box constraints (BoxConstraint ACTIVE_SET / FULL_SET) in the SQP
(TrajoptMPCReference.py:238-248, 273-294; TrajoptConstraint.py:53-130, 210-293).

* Against the reference's own solves (tests/golden/hard_*.npz: 1-link arm, torque
  limits -- the only size the reference's BoxConstraint runs): exit
  code, SQP iterations, per-QP PCG counts (with the reference's nx-aligned
  preconditioner blocks that the appended rows shift), the alpha path, the
  constraint-violation trace and the trajectories.  FULL_SET with PCG: the
  reference raises LinAlgError (singular S), the drop-in raises too.
  The active set of every QP (per-knot bitmasks) equals the one read back from the
  reference's own C.
* Against the oracle's elementwise vector semantics (oracle/hard.py) for n > 1 and
  two limit types at once, the oracle's PCG in the GPU's canonical summation order
  (on these systems two valid orders stop up to 5 iterations apart on the same S,
  oracle/hard.py): every integer exact -- exit codes, SQP iterations, alpha path,
  per-QP PCG counts, per-QP active sets, singular flags.
* QP by QP (tmpc_qp_batch + tmpc_qp_hard_info): at every iterate of the oracle's SQP
  the active sets exactly; S and gamma to 1e-10; the canonical PCG on the GPU's own S
  reproduces the GPU's PCG count exactly and its lambda bit for bit.  This is the
  parity statement for runs whose SQP-level path is rounding-decided: after a full
  step, entries land exactly on a bound and whether the next QP holds them active is
  decided by the last bit (pendulum, iterate 3: u[8..10] = 7 - 8.9e-16, 7,
  7 + 8.9e-16), so two correct solvers may take different active sets from there.
* The GPU's banded PCG on the oracle's own S (tmpc_hard_pcg_batch): counts exact,
  lambda bitwise.
* Singular S (xs outside a state limit; FULL_SET): lstsq's minimum-norm answer and the
  singular flag, methods S and N.
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
    # the active set of every QP, read back from the reference's own C (torque limits of the 1-link arm:
    # bit 4 = lower bound violated, bit 5 = upper; knot by knot)
    ref_masks = [[0] * N for _ in range(len(d["C_rows"]))]
    for q, k, sg in zip(d["act_qp"], d["act_knot"], d["act_sign"]):
        ref_masks[int(q)][int(k)] |= 1 << (4 if int(sg) > 0 else 5)
    assert solver.active_sets == ref_masks
    tr = solver.trace
    if "tr_singular" in d:
        assert [t["singular"] for t in tr] == list(d["tr_singular"].astype(bool))
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
    ("arm3", 12, 2, "N", {"velocity": (-0.5, 0.5, "FULL_SET")}),
    ("arm2", 16, 3, "PCG-SS", {"torque": (-0.4, 0.4, "ACTIVE_SET")}),
]


def _hard_spec(con, n, spec):
    for kind, (lb, ub, mode) in spec.items():
        getattr(con, f"set_{kind}_limits")([ub] * n, [lb] * n, mode)


@pytest.mark.parametrize("name,N,B,method,spec", CASES,
                         ids=[f"{c[0]}-N{c[1]}-{c[3]}-{'+'.join(c[4])}" for c in CASES])
def test_hard_batch_matches_oracle(name, N, B, method, spec):
    """Elementwise vector semantics (oracle/hard.py), problem by problem, against the oracle's SQP:
    exit code, SQP iterations, the alpha path, every QP's active set (per-knot bitmasks) and singular
    flag identical; trajectories at 1e-5.

    PCG counts: on these systems the count is decided by the last bits of S -- arm3 seed 400's QP 1
    stops at 66 iterations on the oracle's S in NumPy's order, at 67 on the same S in the canonical
    order, and the GPU (its own S: blockwise formation, ABA dynamics, ~1e-13 apart) takes 67 -- so
    counts are compared where the inputs are identical, with no tolerance: every QP of the GPU's own
    SQP is replayed at the GPU's iterate (x_j, u_j from the same solve stopped after j iterations,
    rho_j from the trace's schedule, the SQP's xs) through tmpc_qp_batch, which must take the trace's PCG count,
    and the canonical-order PCG (oracle/hard.py) on that QP's S must take it too, with the GPU's
    lambda bit for bit."""
    from oracle import hard as ohard
    from oracle import sqp as osqp
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant,
                                         planar_arm_urdf)
    m = arm_model(name)
    n = m.n
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
    con = TrajoptConstraint(n, n, n, N)
    _hard_spec(con, n, spec)
    solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(n)), con)
    xs, us = zip(*[osqp.initial_problem(m, N, 0.1, 400 + i) for i in range(B)])
    r = solver.SQP_batch(np.array(xs), np.array(us), N, 0.1, method, {}, hard_active=True)
    hard = ohard.HardConstraints([ohard.HardLimit(k, n, lb, ub, mode) for k, (lb, ub, mode) in spec.items()])
    for i in range(B):
        o = osqp.sqp(m, osqp.QuadCost(*quad_cost_arrays(n)), xs[i], us[i], N, 0.1, method, {}, hard=hard,
                     order="canonical")
        got = (int(r["exit_sqp"][i]), int(r["sqp_iter"][i]))
        assert got == (o["exit_sqp"], o["sqp_iter"]), (i, got)
        nq = got[1] + (1 if got[0] == 3 else 0)
        assert list(r["trace"]["alpha"][i, 1:nq + 1]) == [t["alpha"] for t in o["trace"][1:]], i
        masks = [[int(v) for v in r["trace"]["hard_active"][i, q + 1]] for q in range(nq)]
        assert masks == o["active_masks"], i
        assert [bool(v) for v in r["trace"]["singular"][i, 1:nq + 1]] == o["singular"], i
        scale = max(1.0, float(np.max(np.abs(o["x"]))))
        assert float(np.max(np.abs(r["x"][i] - o["x"]))) < 1e-5 * scale, i
    if method.startswith("PCG"):
        _replay_pcg_counts(solver, r, np.array(xs), np.array(us), N, method, hard, n)


def _replay_pcg_counts(solver, r, x0s, u0s, N, method, hard, n, base_opts=None):
    from oracle import hard as ohard
    nx = 2 * n
    B = x0s.shape[0]
    nqs = [int(r["sqp_iter"][i]) + (1 if int(r["exit_sqp"][i]) == 3 else 0) for i in range(B)]
    base_opts = dict(base_opts or {})
    opts = dict(base_opts)
    solver.set_default_options(opts)
    ctx = solver._context(opts)
    # rho of each QP: the trace row holds rho before check_for_exit_or_error's increase on a failed line
    # search (:463-481, as the reference's trace), so replay the schedule from the succeeded flags
    rho_seq = []
    for i in range(B):
        rho, drho, seq = opts["rho_init_SQP_DDP"], 1.0, []
        f = float(opts["rho_factor_SQP_DDP"])
        for j in range(nqs[i]):
            seq.append(rho)
            if r["trace"]["succeeded_line_search"][i, j + 1]:
                drho = min(drho / f, 1.0 / f)
            else:
                drho = max(drho * f, f)
            rho = max(rho * drho, opts["rho_min_SQP_DDP"])
        rho_seq.append(seq)
    for j in range(max(nqs)):
        live = [i for i in range(B) if j < nqs[i]]
        if j == 0:
            xj, uj = x0s[live], u0s[live]
        else:   # the GPU's own iterate j: the same solve, stopped after j iterations
            rj = solver.SQP_batch(x0s, u0s, N, 0.1, method, dict(base_opts, max_iter_SQP_DDP=j))
            xj, uj = rj["x"][live], rj["u"][live]
        rho = np.array([rho_seq[i][j] for i in live])
        ctx = solver._context(dict(opts))
        q = ctx.qp_batch(xj, uj, N, 0.1, rho, method, want_blocks=False, xs=x0s[live][:, :, 0])
        info = ctx.qp_hard_info(len(live), N)
        W = info["W"]
        for a, i in enumerate(live):
            want = int(r["trace"]["pcg_iters"][i, j + 1])
            assert int(q["pcg_iters"][a]) == want, (i, j, int(q["pcg_iters"][a]), want)
            assert [int(v) for v in info["active"][a]] == [int(v) for v in r["trace"]["hard_active"][i, j + 1]]
            D = int(info["dim"][a])
            S_g = _unband(info["S_band"][a], W, D)
            lam_c, it_c = ohard.pcg_canonical(S_g, info["gamma"][a, :D], nx, method[4:],
                                              opts["exit_tolerance_linSys"], opts["max_iter_linSys"])
            assert it_c == want, (i, j, it_c, want)
            dyn, hrows = _row_layout(hard, xj[a], uj[a], N, nx)
            nz = (nx + n) * (N - 1) + nx
            assert np.array_equal(q["dxul"][a][nz:], lam_c[dyn]), (i, j)


def test_hard_constraints_reject_ilqr():
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant, _native,
                                         planar_arm_urdf)
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(2)})
    con = TrajoptConstraint(2, 2, 2, 8)
    con.set_torque_limits([1.0] * 2, [-1.0] * 2, "ACTIVE_SET")
    solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(2)), con)
    with pytest.raises(_native.NativeError, match="iLQR"):
        solver.iLQR(np.zeros((4, 8)), np.zeros((2, 7)), 8, 0.1, {})


def _row_layout(hard, x, u, N, nx):
    """(dynamics / initial-state row indices in knot order, [(row, knot, slot)] of the hard rows) in the
    reference's row order R_0 | R_1 H_0 | ... (oracle/hard.py kkt_dense); slot = t * 2n + e"""
    n = nx // 2
    modes = {lim.kind: lim.mode for lim in hard.limits}
    kinds = ("joint", "velocity", "torque")
    dyn = list(range(nx))
    hrows = []
    r = nx
    for k in range(N):
        if k < N - 1:
            dyn += list(range(r, r + nx))
            r += nx
        rows = hard.rows(x[:, k], u[:, k] if k < N - 1 else None, k, N)
        pos = {}
        for j, (col, sign, _) in enumerate(rows):
            t, i = divmod(col, n)
            if modes[kinds[t]] == "FULL_SET":   # every entry has a row, in order lb 0..n-1, ub 0..n-1
                e = pos.get(t, 0)
                pos[t] = e + 1
            else:
                e = i if sign > 0 else n + i
            hrows.append((r + j, k, t * 2 * n + e))
        r += len(rows)
    return dyn, hrows


def _band(S, W):
    D = S.shape[0]
    Sb = np.zeros((D, 2 * W + 1))
    for o in range(2 * W + 1):
        a = np.arange(D)
        c = a - W + o
        ok = (c >= 0) & (c < D)
        Sb[a[ok], o] = S[a[ok], c[ok]]
    return Sb


def _unband(Sb, W, D):
    S = np.zeros((D, D))
    for o in range(2 * W + 1):
        a = np.arange(D)
        c = a - W + o
        ok = (c >= 0) & (c < D)
        S[a[ok], c[ok]] = Sb[a[ok], o]
    return S


QP_CASES = [
    ("pendulum", 20, "S", {"torque": (-7.0, 7.0, "ACTIVE_SET")}),
    ("pendulum", 20, "PCG-SS", {"torque": (-7.0, 7.0, "ACTIVE_SET")}),
    ("arm3", 12, "PCG-SS", {"torque": (-0.3, 0.3, "ACTIVE_SET"), "velocity": (-0.6, 0.6, "ACTIVE_SET")}),
    ("arm3", 12, "PCG-BJ", {"torque": (-0.3, 0.3, "ACTIVE_SET"), "velocity": (-0.6, 0.6, "ACTIVE_SET")}),
    ("arm3", 12, "S", {"velocity": (-0.5, 0.5, "FULL_SET")}),
    ("arm2", 16, "PCG-J", {"torque": (-0.4, 0.4, "ACTIVE_SET"), "joint": (-1.0, 1.0, "ACTIVE_SET")}),
]


def _qp_problem(name, N, spec):
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
        model = plant.model
    else:
        model = arm_model(name)
        n = model.n
        plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
        Q, QF, R, xg = quad_cost_arrays(n)
        x0, u0 = osqp.initial_problem(model, N, 0.1, 430)
        opts = {}
    con = TrajoptConstraint(n, n, n, N)
    _hard_spec(con, n, spec)
    solver = TrajoptMPCReference(plant, QuadraticCost(Q, QF, R, xg), con)
    hard = ohard.HardConstraints([ohard.HardLimit(k, n, lb, ub, mode) for k, (lb, ub, mode) in spec.items()])
    return solver, model, hard, osqp.QuadCost(Q, QF, R, xg), x0, u0, opts, n


@pytest.mark.parametrize("name,N,method,spec", QP_CASES,
                         ids=[f"{c[0]}-N{c[1]}-{c[2]}-{'+'.join(c[3])}" for c in QP_CASES])
def test_hard_qp_matches_oracle_at_every_iterate(name, N, method, spec):
    """Every QP of one oracle SQP run, batched as B problems on the GPU (tmpc_qp_batch +
    tmpc_qp_hard_info), on identical (x, u, rho):
      * the active set of every knot (bitmasks) and the Schur dimension: identical;
      * the GPU's banded S and gamma against the oracle's dense -C G^-1 C^T, c - C G^-1 g: 1e-10 relative
        (two formation orders; A, B from two dynamics implementations);
      * PCG: the oracle's canonical-order PCG (oracle/hard.py pcg_canonical) on the GPU's own S and
        gamma -- identical inputs -- stops at the GPU's PCG count EXACTLY and returns the GPU's lambda
        (dynamics rows and hard rows) BIT FOR BIT;
      * method S: dxul against the oracle's dense solve at 1e-9; the singular flag identical;
      * the step dxu against the exact QP solution within 100x of the oracle's own PCG answer's distance."""
    from oracle import hard as ohard
    from oracle import sqp as osqp
    solver, model, hard, oc, x0, u0, opts, n = _qp_problem(name, N, spec)
    nx = 2 * n
    o = osqp.sqp(model, oc, x0, u0, N, 0.1, method, dict(opts), hard=hard, order="canonical")
    its = o["iterates"]
    assert len(its) == len(o["dxul"]) >= 2
    full = dict(opts)
    solver.set_default_options(full)
    ctx = solver._context(full)
    xs = np.array([x for x, _, _ in its])
    us = np.array([u for _, u, _ in its])
    rho = np.array([r for _, _, r in its])
    B = len(its)
    # the SQP's xs: the QP's initial-state row is x_0 - xs
    r = ctx.qp_batch(xs, us, N, 0.1, rho, method, want_blocks=False, xs=np.repeat(x0[:, 0][None], B, 0))
    info = ctx.qp_hard_info(B, N)
    W = info["W"]
    nz = (nx + n) * (N - 1) + nx
    o_opts = osqp.default_options(opts)
    for i, (x, u, rho_i) in enumerate(its):
        assert [int(v) for v in info["active"][i]] == o["active_masks"][i], i
        dyn, hrows = _row_layout(hard, x, u, N, nx)
        G, g, Cm, cc = ohard.kkt_dense(model, oc, x, u, x0[:, 0], N, 0.1, hard)
        D = Cm.shape[0]
        assert int(info["dim"][i]) == D, i
        Gr = G + rho_i * np.eye(G.shape[0])
        invG = np.linalg.inv(Gr)
        S_o = -Cm @ (invG @ Cm.T)
        gam_o = cc - Cm @ (invG @ g)
        S_g = _unband(info["S_band"][i], W, D)
        gam_g = info["gamma"][i, :D]
        assert float(np.max(np.abs(S_g - S_o))) <= 1e-10 * float(np.max(np.abs(S_o))), i
        assert float(np.max(np.abs(gam_g - gam_o))) <= 1e-10 * max(1.0, float(np.max(np.abs(gam_o)))), i
        got = r["dxul"][i]
        lam_dyn = got[nz:]
        lam_hard = np.array([info["lambda_hard"][i, k, sl] for _, k, sl in hrows])
        ref = o["dxul"][i]
        sc = max(1.0, float(np.max(np.abs(ref[:nz]))))
        if method == "S":
            assert bool(info["singular"][i]) == o["singular"][i], i
            sl = max(1.0, float(np.max(np.abs(ref[nz:]))))
            assert float(np.max(np.abs(got[:nz] - ref[:nz]))) < 1e-9 * sc, i
            assert float(np.max(np.abs(lam_dyn - ref[nz:][dyn]))) < 1e-9 * sl, i
            if hrows:
                assert float(np.max(np.abs(lam_hard - ref[nz:][[a for a, _, _ in hrows]]))) < 1e-9 * sl, i
            continue
        # identical inputs: the canonical-order PCG on the GPU's own S / gamma is the GPU's PCG, bit for bit
        lam_c, it_c = ohard.pcg_canonical(S_g, gam_g, nx, method[4:], o_opts["exit_tolerance_linSys"],
                                          o_opts["max_iter_linSys"])
        assert int(r["pcg_iters"][i]) == it_c, (i, int(r["pcg_iters"][i]), it_c)
        assert np.array_equal(lam_dyn, lam_c[dyn]), i
        assert np.array_equal(lam_hard, lam_c[[a for a, _, _ in hrows]]), i
        # the step against the exact QP solution, relative to the oracle's own truncated PCG answer: the
        # two PCG paths start from S 1e-13 apart and stop anywhere inside the |nu| < 1e-6 region of these
        # erratically converging systems (measured up to 11x apart, arm3 PCG-SS iterate 1), so 100x
        ex, _, _ = ohard.solve_qp_dense(G, g, Cm, cc, rho_i, "S", o_opts, nx)
        e_ref = float(np.max(np.abs(ref[:nz] - ex[:nz])))
        e_got = float(np.max(np.abs(got[:nz] - ex[:nz])))
        assert e_got <= 100 * e_ref + 1e-9 * sc, (i, e_got, e_ref)


PCG_CASES = [("arm3", 12, "BJ", 400), ("arm3", 12, "SS", 400), ("arm3", 12, "J", 401), ("arm2", 16, "0", 430)]


@pytest.mark.parametrize("name,N,ptype,seed", PCG_CASES, ids=[f"{c[0]}-{c[2]}-s{c[3]}" for c in PCG_CASES])
def test_hard_pcg_on_oracle_S_is_exact(name, N, ptype, seed):
    """The oracle's own hard-row S and gamma (the reference's dense formation, every QP of an oracle SQP
    run) fed to the GPU's banded PCG (tmpc_hard_pcg_batch): PCG counts identical to the oracle's
    canonical-order PCG and lambda bit for bit.  The seeds include the QPs whose count the summation
    order itself decides (arm3 seed 400: NumPy's order and the canonical one stop up to 5 iterations
    apart on the same S, oracle/hard.py), i.e. exactness here is a statement about identical
    arithmetic, not about well-conditioned systems."""
    from oracle import hard as ohard
    from oracle import sqp as osqp
    from trajoptmpcreference_amd import _native
    m = arm_model(name)
    n = m.n
    nx = 2 * n
    spec = {"torque": (-0.3, 0.3, "ACTIVE_SET"), "velocity": (-0.6, 0.6, "ACTIVE_SET")}
    hard = ohard.HardConstraints([ohard.HardLimit(k, n, lb, ub, mode) for k, (lb, ub, mode) in spec.items()])
    cost = osqp.QuadCost(*quad_cost_arrays(n))
    x0, u0 = osqp.initial_problem(m, N, 0.1, seed)
    o = osqp.sqp(m, cost, x0, u0, N, 0.1, "PCG-" + ptype, {}, hard=hard, order="canonical")
    Ss, gs, dims = [], [], []
    for x, u, rho in o["iterates"]:
        G, g, C, c = ohard.kkt_dense(m, cost, x, u, x0[:, 0], N, 0.1, hard)
        invG = np.linalg.inv(G + rho * np.eye(G.shape[0]))
        Ss.append(-C @ (invG @ C.T))
        gs.append(c - C @ (invG @ g))
        dims.append(C.shape[0])
    dmax = max(dims)
    W = max(int(np.max(np.abs(np.subtract(*np.nonzero(S))))) for S in Ss)
    Sb = np.zeros((len(Ss), dmax, 2 * W + 1))
    gb = np.zeros((len(Ss), dmax))
    for i, (S, gm) in enumerate(zip(Ss, gs)):
        Sb[i, :len(gm)] = _band(S, W)
        gb[i, :len(gm)] = gm
    ctx = _native.default_context(0)
    ctx.set_model(m)
    ctx.reset_stats()
    lam, it = ctx.hard_pcg_batch(Sb, gb, dims, nx, ptype)
    for i, (S, gm) in enumerate(zip(Ss, gs)):
        lam_c, it_c = ohard.pcg_canonical(S, gm, nx, ptype, 1e-6, 100)
        assert int(it[i]) == it_c, (i, int(it[i]), it_c)
        assert np.array_equal(lam[i, :len(gm)], lam_c), i
    # the kernel's own algorithmic-byte count (the hard bench line's roofline), exactly
    assert ctx.kernel_bytes("hard_pcg") == _hard_pcg_bytes(Ss, it, nx, ptype, dmax)


LARGE_CASES = [(ptype, 12, (1530, 1100, 700), "arm6fix") for ptype in ("SS", "BJ", "J")] + \
    [("SS", 14, (3000, 2100), "arm7"), ("SS", 14, (4000, 3100), "arm7"), ("BJ", 14, (4090,), "arm7")]


@pytest.mark.parametrize("ptype,nx,dims_,model", LARGE_CASES,
                         ids=[f"{c[0]}-nx{c[1]}-D{c[2][0]}" for c in LARGE_CASES])
def test_hard_pcg_large_banded_is_exact(ptype, nx, dims_, model):
    """Schur dimensions past one 1024-row slot and past the LDS block cache (D = 1530: 94 of 127 diagonal
    blocks fit, the rest stream from HBM; D = 1100 and 700 alongside, all cached; D = 3000 at nx = 14:
    three row slots, 35 of 214 diagonal blocks cached; D = 4000 and 4090 at nx = 14: the four-slot instance
    k_hard_pcg<14, 4> at the edge of the LDS budget, 9 blocks cached), trailing partial blocks
    (1530 mod 12 = 6, 3000 mod 14 = 4, 4000 mod 14 = 10 unpreconditioned rows): counts and lambda bit for
    bit against pcg_canonical, and the kernel's byte count exactly."""
    from oracle import hard as ohard
    from trajoptmpcreference_amd import _native
    W = 30
    rng = np.random.default_rng(7)
    Ss, gs = [], []
    for D in dims_:
        M = np.zeros((D, D))
        for o in range(-W // 2, W // 2 + 1):
            M += np.diag(rng.uniform(-1.0, 1.0, D - abs(o)), o)
        Ss.append(-(M @ M.T + 2.0 * np.eye(D)))
        gs.append(rng.uniform(-1.0, 1.0, D))
    dims = [len(g) for g in gs]
    dmax = max(dims)
    Sb = np.zeros((len(Ss), dmax, 2 * W + 1))
    gb = np.zeros((len(Ss), dmax))
    for i, (S, gm) in enumerate(zip(Ss, gs)):
        Sb[i, :len(gm)] = _band(S, W)
        gb[i, :len(gm)] = gm
    ctx = _native.default_context(0)
    ctx.set_model(arm_model(model))
    ctx.reset_stats()
    lam, it = ctx.hard_pcg_batch(Sb, gb, dims, nx, ptype, tol=1e-10, max_iter=200)
    for i, (S, gm) in enumerate(zip(Ss, gs)):
        lam_c, it_c = ohard.pcg_canonical(S, gm, nx, ptype, 1e-10, 200)
        assert 5 < it_c < 200, it_c
        assert int(it[i]) == it_c, (i, int(it[i]), it_c)
        assert np.array_equal(lam[i, :len(gm)], lam_c), i
    assert ctx.kernel_bytes("hard_pcg") == _hard_pcg_bytes(Ss, it, nx, ptype, dmax)


def _hard_pcg_bytes(Ss, iters, nx, ptype, dmax):
    """8 B x (2 D + it x band entries + (it + 1) x streamed preconditioner entries + setup blocks) per
    problem; band entries: each row's first..last nonzero column (with the diagonal), the range the kernel
    visits; streamed preconditioner entries: the distinct blocks one P^-1 r needs (SS: nb diagonal + nb - 1
    stair) less those the kernel keeps in LDS -- as many as fit in the 160 KB after its vectors, diagonal
    blocks first (tmpc_hard.hip hard_pcg_cache_offset)."""
    slots = -(-dmax // 1024)
    # tmpc_hard.hip hard_pcg_reg_diag (slot 0, in registers; TMPC_HARD_REG, a build constant)
    reg = int(os.environ.get("TMPC_TEST_HARD_REG", "24"))
    REG = (16 if nx <= 4 else (reg - 4 if nx >= 14 or nx == 8 else reg)) - (8 if slots >= 3 else 0)
    tot = 0.0
    for S, it in zip(Ss, iters):
        D = S.shape[0]
        nnz, nnz_reg = 0, 0
        for a in range(D):
            nzc = np.nonzero(S[a])[0]
            width = max(a, int(nzc.max(initial=a))) - min(a, int(nzc.min(initial=a))) + 1
            streamed = max(0, width - REG) if a < 1024 else width
            nnz += streamed
            nnz_reg += width - streamed
        nb, b2 = D // nx, nx * nx
        offset = max(2 * D + 2 * max(D - 1024, 0), 4 * (b2 + 2 * nx)) + 32 + (D + 2 * slots * 16 + 1) // 2
        offset += offset & 1   # 16-byte aligned
        ncap = max(0, 160 * 1024 // 8 - offset) // b2
        ncd = min(nb, ncap) if ptype in ("BJ", "SS") else 0
        ncl = min(nb - 1, ncap - ncd) if ptype == "SS" and nb > 1 else 0
        # setup: the band blocks read, and the HBM writes of the blocks the LDS cache does not hold
        pnnz, setup = {"0": (0, 0), "J": (D, 0), "BJ": ((nb - ncd) * b2, (nb + 2 * (nb - ncd)) * b2),
                       "SS": ((2 * nb - 1 - ncd - ncl) * b2,
                              (2 * nb - 1 + 2 * (nb - ncd) + (nb - 1 - ncl)) * b2) if nb else (0, 0)}[ptype]
        tot += 8.0 * (2.0 * D + int(it) * nnz + (int(it) + 1.0) * pnnz + setup + nnz_reg)
    return tot


def test_hard_singular_duplicate_rows():
    """xs outside a velocity limit: the knot-0 hard row duplicates the initial-state row (up to sign),
    so S is singular in exact arithmetic.  The reference's np.linalg.solve raises or not
    depending on the elimination's rounding; the build defines the answer as lstsq's minimum-norm
    solution (its fallback, TrajoptMPCReference.py:431-436) with `singular` set (oracle/hard.py
    structurally_singular), for methods S and N alike.  QP level: dxul against the oracle's lstsq
    answer at 1e-9 on identical inputs, finite everywhere; SQP level: exit code, iterations, alpha
    path, active sets and singular flags identical, trajectories at 1e-6."""
    from oracle import hard as ohard
    from oracle import rbd
    from oracle import sqp as osqp
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant,
                                         planar_arm_urdf)
    m = arm_model("arm3")
    n, N = 3, 8
    nx = 2 * n
    x0, u0 = osqp.initial_problem(m, N, 0.1, 5)
    x0[n:, 0] = [0.9, -0.2, 0.1]
    for k in range(N - 1):
        x0[:, k + 1] = rbd.euler(m, x0[:, k][None], u0[:, k][None], 0.1)[0]
    spec = {"velocity": (-0.5, 0.5, "ACTIVE_SET")}
    hard = ohard.HardConstraints([ohard.HardLimit("velocity", n, -0.5, 0.5, "ACTIVE_SET")])
    cost = osqp.QuadCost(*quad_cost_arrays(n))
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
    nz = (nx + n) * (N - 1) + nx
    for method in ("S", "N"):
        con = TrajoptConstraint(n, n, n, N)
        _hard_spec(con, n, spec)
        solver = TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(n)), con)
        o = osqp.sqp(m, cost, x0, u0, N, 0.1, method, {}, hard=hard)
        assert all(o["singular"]) and o["active_masks"][0][0] != 0
        x, u, ex, _, _, it = solver.SQP(x0, u0, N, 0.1, method, {})
        assert (ex, it) == (o["exit_sqp"], o["sqp_iter"]), method
        tr = solver.trace
        assert [t["alpha"] for t in tr] == [t["alpha"] for t in o["trace"]], method
        assert all(t["singular"] for t in tr[1:]) and solver.singular, method
        assert solver.active_sets == o["active_masks"], method
        assert np.max(np.abs(x - o["x"])) < 1e-6 * max(1.0, float(np.max(np.abs(o["x"])))), method
        # QP level on the oracle's iterates
        its = o["iterates"]
        opts = {}
        solver.set_default_options(opts)
        ctx = solver._context(opts)
        xs = np.array([a for a, _, _ in its])
        r = ctx.qp_batch(xs, np.array([b for _, b, _ in its]), N, 0.1, np.array([c for _, _, c in its]), method,
                         want_blocks=False, xs=np.repeat(x0[:, 0][None], len(its), 0))
        info = ctx.qp_hard_info(len(its), N)
        assert np.all(info["singular"] == 1)
        for i in range(len(its)):
            got, ref = r["dxul"][i], o["dxul"][i]
            assert np.all(np.isfinite(got))
            dyn, _ = _row_layout(hard, its[i][0], its[i][1], N, nx)
            sc = max(1.0, float(np.max(np.abs(ref[:nz]))))
            assert float(np.max(np.abs(got[:nz] - ref[:nz]))) < 1e-9 * sc, (method, i)
            sl = max(1.0, float(np.max(np.abs(ref[nz:]))))
            assert float(np.max(np.abs(got[nz:] - ref[nz:][dyn]))) < 1e-9 * sl, (method, i)


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
