#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE
(VCA-EPFL/TrajoptMPCReference, read-only at /root/reference) in this container.

This script is test infrastructure.  It is the only place that imports the
reference, it runs only here (the reference does not exist on the GPU box),
and what it writes is data: inputs and the reference's outputs, as .npz.

Import recipe:
  * /root/reference on sys.path, PYTHONDONTWRITEBYTECODE=1 (read-only tree);
  * a one-line ``bs4`` stub ahead on sys.path for the dead import at
    GRiD/URDFParser/URDFParser.py:212;
  * arm6.urdf is malformed (joint6 repeats joint5's parent/child,
    models/arm6.urdf:75-80); we feed the reference a corrected copy
    (joint6: link5 -> link6) written to a temp dir;
  * QuadraticCost methods do not accept the iter_* kwargs SQP passes
    (TrajoptCost.py:49,58,71 vs TrajoptMPCReference.py:218-219);
    we subclass it with pass-through signatures (public plugin subclassing).

Usage:  python tests/golden/make_golden.py [--quick]
"""
import argparse
import copy
import multiprocessing as mp
import os
import sys
import tempfile
import time

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
_STUB_DIR = None


def _setup_reference():
    global _STUB_DIR
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    if _STUB_DIR is None:
        _STUB_DIR = tempfile.mkdtemp(prefix="tmpc_stub_")
        with open(os.path.join(_STUB_DIR, "bs4.py"), "w") as f:
            f.write("BeautifulSoup = None\n")
    for p in (REF, _STUB_DIR):
        if p not in sys.path:
            sys.path.insert(0, p)


def model_path(name):
    """arm2/arm3 as shipped; arm6 with the 2-line joint6 fix."""
    src = os.path.join(REF, "models", name.replace("fix", "") + ".urdf")
    if not name.endswith("fix"):
        return src
    text = open(src).read()
    head, tail = text.split('<joint name="joint6"', 1)
    tail = tail.replace('<parent link="link4"/>', '<parent link="link5"/>', 1)
    tail = tail.replace('<child link="link5"/>', '<child link="link6"/>', 1)
    d = tempfile.mkdtemp(prefix="tmpc_urdf_")
    p = os.path.join(d, name + ".urdf")
    with open(p, "w") as f:
        f.write(head + '<joint name="joint6"' + tail)
    return p


def make_plant(name):
    _setup_reference()
    from TrajoptPlant import URDFPlant
    return URDFPlant(options={"path_to_urdf": model_path(name), "overloading": False})


def make_cost(nx, nu):
    _setup_reference()
    from TrajoptCost import QuadraticCost

    class PassThroughQuadraticCost(QuadraticCost):
        # accepts the iter_* arguments SQP passes
        def value(self, x, u=None, timestep=None, *a, **k):
            return QuadraticCost.value(self, x, u, timestep)

        def gradient(self, x, u=None, timestep=None, *a, **k):
            return QuadraticCost.gradient(self, x, u, timestep)

        def hessian(self, x, u=None, timestep=None, *a, **k):
            return QuadraticCost.hessian(self, x, u, timestep)

    return PassThroughQuadraticCost(np.eye(nx), 100.0 * np.eye(nx), 0.1 * np.eye(nu), np.zeros(nx))


def initial_problem(plant, N, dt, seed):
    """The §8d workload: q0 ~ U(-1,1)^n from default_rng(seed), qd0 = 0,
    x = Euler rollout of u = 0, u = 0."""
    n = plant.get_num_pos()
    rng = np.random.default_rng(seed)
    x = np.zeros((2 * n, N))
    x[:n, 0] = rng.uniform(-1.0, 1.0, n)
    u = np.zeros((n, N - 1))
    for k in range(N - 1):
        x[:, k + 1] = plant.integrator(x[:, k], u[:, k], dt)
    return x, u


# ---------------------------------------------------------------- model + dynamics
def gen_model_and_dynamics(name, K=32, seed=1234):
    plant = make_plant(name)
    robot = plant.robot
    rbd = plant.rbdReference
    n = robot.get_num_pos()
    qs = np.array([[0.0] * n, [0.3] * n, [-1.7] * n, list(np.linspace(-3.0, 3.0, n)), list(np.linspace(2.5, -0.4, n))])
    X = np.zeros((len(qs), n, 6, 6))
    for a, q in enumerate(qs):
        for j in range(n):
            X[a, j] = np.asarray(robot.get_Xmat_Func_by_id(j)(q[j]), dtype=float)
    np.savez_compressed(
        os.path.join(OUT, f"model_{name}.npz"),
        parent=np.array([robot.get_parent_id(j) for j in range(n)], dtype=np.int32),
        S=np.array([robot.get_S_by_id(j) for j in range(n)], dtype=float),
        I=np.array([robot.get_Imat_by_id(j) for j in range(n)], dtype=float),
        qs=qs, X=X)

    from GRiD.util import util
    q0, qd0, u0, _ = util.initializeValues(robot, MATCH_CPP_RANDOM=True)
    rng = np.random.default_rng(seed)
    xs = [np.concatenate([q0, qd0])]
    us = [u0]
    for _ in range(K - 1):
        xs.append(np.concatenate([rng.uniform(-np.pi, np.pi, n), rng.uniform(-2, 2, n)]))
        us.append(rng.uniform(-1.5, 1.5, n))
    xs = np.array(xs)
    us = np.array(us)
    dt = 0.1
    out = {k: [] for k in ["qdd", "dqdd", "xnext", "A", "B", "c", "Minv", "dc_du"]}
    for x, u in zip(xs, us):
        q, qd = x[:n], x[n:]
        out["qdd"].append(plant.forward_dynamics(x, u))
        out["dqdd"].append(plant.forward_dynamics_gradient(x, u))
        out["xnext"].append(plant.integrator(x, u, dt))
        A, B = plant.integrator(x, u, dt, return_gradient=True)
        out["A"].append(A)
        out["B"].append(B)
        c, _, _, _ = rbd.rnea(q, qd, None, -9.81)
        out["c"].append(c)
        out["Minv"].append(rbd.minv(q))
        out["dc_du"].append(rbd.rnea_grad(q, qd, out["qdd"][-1], -9.81))
    np.savez_compressed(os.path.join(OUT, f"dyn_{name}.npz"), x=xs, u=us, dt=dt,
                        **{k: np.array(v) for k, v in out.items()})
    print(f"[golden] model/dyn {name}: n={n} K={K}", flush=True)


# ---------------------------------------------------------------- one QP
def _blocks(M, nx, N):
    d = np.array([M[k * nx:(k + 1) * nx, k * nx:(k + 1) * nx] for k in range(N)])
    lo = np.array([M[(k + 1) * nx:(k + 2) * nx, k * nx:(k + 1) * nx] for k in range(N - 1)])
    up = np.array([M[k * nx:(k + 1) * nx, (k + 1) * nx:(k + 2) * nx] for k in range(N - 1)])
    return d, lo, up


def gen_qp(name, N, seed=0, dt=0.1, rho=1e-3):
    _setup_reference()
    from TrajoptMPCReference import TrajoptMPCReference
    import importlib
    PCG = importlib.import_module("GBD-PCG-Python").PCG
    plant = make_plant(name)
    n = plant.get_num_pos()
    nx, nu = 2 * n, n
    cost = make_cost(nx, nu)
    x, u = initial_problem(plant, N, dt, seed)
    xs = copy.deepcopy(x[:, 0])
    solver = TrajoptMPCReference(plant, cost)
    G, g, C, c = solver.formKKTSystemBlocks(x, u, xs, N, dt)
    Ak = np.array([d["value"] for d in solver.saved_Ak])
    Bk = np.array([d["value"] for d in solver.saved_Bk])
    G = G + rho * np.eye(G.shape[0])
    invG = np.linalg.inv(G)
    S = -np.matmul(C, np.matmul(invG, C.T))
    gamma = c - np.matmul(C, np.matmul(invG, g))
    rec = dict(x=x, u=u, rho=rho, dt=dt, g=g[:, 0], c=c[:, 0], A=Ak, B=Bk, gamma=gamma[:, 0])
    rec["S_diag"], rec["S_lo"], rec["S_up"] = _blocks(S, nx, N)
    l_direct = np.linalg.solve(S, gamma)
    rec["lam_direct"] = l_direct[:, 0]
    rec["dxul_direct"] = np.vstack((np.matmul(invG, g - np.matmul(C.T, l_direct)), l_direct))[:, 0]
    for p in ["J", "BJ", "SS", "0"]:
        opts = {"exit_tolerance": 1e-6, "max_iter": 100, "DEBUG_MODE": False, "RETURN_TRACE": False,
                "preconditioner_type": p}
        pcg = PCG(S, gamma, nx, N, options=opts)
        lam, (tr_nu, tr_res) = pcg.solve()
        P = pcg.Pinv
        rec[f"P_{p}_diag"], rec[f"P_{p}_lo"], rec[f"P_{p}_up"] = _blocks(P, nx, N)
        rec[f"lam_{p}"] = lam[:, 0]
        rec[f"trace_nu_{p}"] = np.array(tr_nu)
        rec[f"trace_res_{p}"] = np.array(tr_res)
        rec[f"iters_{p}"] = len(tr_nu) - 1
        rec[f"dxul_{p}"] = np.vstack((np.matmul(invG, g - np.matmul(C.T, lam)), lam))[:, 0]
        # KKT residual computed the §8d way on the reference's own iterate
        KKT = np.block([[G, C.T], [C, np.zeros((C.shape[0], C.shape[0]))]])
        rec[f"kkt_res_{p}"] = np.max(np.abs(KKT @ rec[f"dxul_{p}"] - np.concatenate([g[:, 0], c[:, 0]])))
    # options['guess'] -> PCG.update_guess (TrajoptMPCReference.py:439-440): a perturbed iterate as the
    # initial x of the SS and BJ solves
    rng = np.random.default_rng(4321)
    guess = rec["lam_SS"] * (1.0 + 0.1 * rng.standard_normal(rec["lam_SS"].shape))
    rec["guess"] = guess
    for p in ["BJ", "SS"]:
        opts = {"exit_tolerance": 1e-6, "max_iter": 100, "DEBUG_MODE": False, "RETURN_TRACE": False,
                "preconditioner_type": p}
        pcg = PCG(S, gamma, nx, N, options=opts)
        pcg.update_guess(guess.copy())
        lam, (tr_nu, tr_res) = pcg.solve()
        rec[f"lam_{p}_guess"] = lam[:, 0]
        rec[f"trace_nu_{p}_guess"] = np.array(tr_nu)
        rec[f"iters_{p}_guess"] = len(tr_nu) - 1
        rec[f"dxul_{p}_guess"] = np.vstack((np.matmul(invG, g - np.matmul(C.T, lam)), lam))[:, 0]
    np.savez_compressed(os.path.join(OUT, f"qp_{name}_N{N}.npz"), **rec)
    print(f"[golden] qp {name} N={N}: iters J/BJ/SS/0 = {rec['iters_J']}/{rec['iters_BJ']}/{rec['iters_SS']}/"
          f"{rec['iters_0']}, guess BJ/SS = {rec['iters_BJ_guess']}/{rec['iters_SS_guess']}", flush=True)


# ---------------------------------------------------------------- UrdfCost
EE_Q = np.eye(4)
EE_QF = 100.0 * np.eye(4)
EE_R = 0.1 * np.eye(2)


def make_ee_cost(plant, xg, QF_start=None):
    _setup_reference()
    from TrajoptCost import UrdfCost
    return UrdfCost(plant, EE_Q.copy(), EE_QF.copy(), EE_R.copy(), np.array(xg, dtype=float), QF_start=QF_start)


def gen_ee_points(K=24, seed=77):
    """UrdfCost value / gradient / hessian and the RBDReference EE kinematics at random arm2 states."""
    plant = make_plant("arm2")
    cost = make_ee_cost(plant, [-1.0, 1.5, 0.0, 0.0], QF_start=20)
    rng = np.random.default_rng(seed)
    X = rng.uniform(-2.0, 2.0, (K, 4))
    U = rng.uniform(-3.0, 3.0, (K, 2))
    ks = rng.integers(0, 30, K)
    term = (np.arange(K) % 4) == 3
    rec = {k: [] for k in ["pos", "J", "Jtot", "dx", "value", "grad", "hess"]}
    rbd = plant.rbdReference
    for i in range(K):
        x, u, k = X[i], (None if term[i] else U[i]), int(ks[i])
        rec["pos"].append(np.asarray(rbd.end_effector_positions(x[:2], cost.offsets), dtype=float).reshape(2))
        rec["J"].append(np.asarray(rbd.Jacobian(x[:2], cost.offsets), dtype=float))
        rec["Jtot"].append(np.asarray(rbd.jacobian_tot_state(x[:2], x[2:], cost.offsets), dtype=float))
        rec["dx"].append(np.asarray(cost.delta_x(x), dtype=float).reshape(4))
        rec["value"].append(float(np.asarray(cost.value(x, u, k)).reshape(())))
        g = np.zeros(6)
        gv = np.asarray(cost.gradient(x, u, k), dtype=float).reshape(-1)
        g[:gv.size] = gv
        rec["grad"].append(g)
        h = np.zeros((6, 6))
        hv = np.asarray(cost.hessian(x, u, k), dtype=float)
        h[:hv.shape[0], :hv.shape[1]] = hv
        rec["hess"].append(h)
    np.savez_compressed(os.path.join(OUT, "ee_arm2_points.npz"), X=X, U=U, k=ks, terminal=term, QF_start=20,
                        xg=np.array([-1.0, 1.5, 0.0, 0.0]), **{k: np.array(v) for k, v in rec.items()})
    print(f"[golden] ee points arm2 K={K}")


def run_ee_sqp(args):
    """examples/twolinks.py (type_cost='urdf', PCG-SS, N=10, dt=0.1, x=u=0, expected_reduction_min=-100):
    the configuration data/4 (xg=[-1,1.5,0,0]) and data/3 (xg=[-1.18,-1.58,0,0]) were recorded with."""
    tag, xg, method = args
    _setup_reference()
    from TrajoptMPCReference import TrajoptMPCReference, SQPSolverMethods
    from overloading import matrix_
    matrix_.iteration = 0
    matrix_.soft_constraint_iteration = 0
    matrix_.line_search_iteration = 0
    plant = make_plant("arm2")
    cost = make_ee_cost(plant, xg)
    N, dt = 10, 0.1
    x0, u0 = np.zeros((4, N)), np.zeros((2, N - 1))
    solver = TrajoptMPCReference(plant, cost)
    m = {"S": SQPSolverMethods.S, "PCG-SS": SQPSolverMethods.PCG_SS, "PCG-BJ": SQPSolverMethods.PCG_BJ}[method]
    opts = {"expected_reduction_min_SQP_DDP": -100, "RETURN_TRACE_SQP": True, "overloading": False}
    import io
    import contextlib
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(copy.deepcopy(x0), copy.deepcopy(u0), N, dt, m,
                                                                     opts)
    wall = time.time() - t0
    tr = solver.trace
    keys = ["iteration", "line_search_iteration", "alpha", "rho", "J", "c", "merit", "D", "reduction_ratio",
            "succeeded_line_search"]
    rec = {"tr_" + k: np.array([np.nan if t[k] is None else float(t[k]) for t in tr]) for k in keys}
    pcg_iters = np.array([len(t[0][0]) - 1 for t in solver.saved_inner_traces], dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, f"ee_sqp_arm2_N10_{tag}_{method}.npz"),
                        x0=x0, u0=u0, x=np.asarray(x), u=np.asarray(u), dt=dt, xg=np.array(xg, dtype=float),
                        expected_reduction_min=-100.0, exit_sqp=exit_sqp, exit_soft=exit_soft,
                        outer_iter=outer_iter, sqp_iter=sqp_iter, pcg_iters=pcg_iters, wall_s=wall, **rec)
    return f"[golden] ee sqp {tag} {method}: exit={exit_sqp} iters={sqp_iter} pcg={list(pcg_iters)} wall={wall:.1f}s"


def gen_ee_recorded():
    """The recorded twolinks runs' final trajectories (data/4, data/3 CSVs: data, read as text)."""
    out = {}
    for tag in ("4", "3"):
        for nm in ("final_traj", "final_input"):
            path = os.path.join(REF, "data", tag, nm + ".csv")
            if os.path.exists(path):
                out[f"d{tag}_{nm}"] = np.loadtxt(path, delimiter=",", skiprows=1)[:, 1:]
    np.savez_compressed(os.path.join(OUT, "ee_arm2_recorded.npz"), **out)
    print(f"[golden] ee recorded: {sorted(out)}")


# ---------------------------------------------------------------- full SQP
def run_sqp(args):
    name, N, seed, method, dt = args
    _setup_reference()
    from TrajoptMPCReference import TrajoptMPCReference, SQPSolverMethods
    from overloading import matrix_
    matrix_.iteration = 0
    matrix_.soft_constraint_iteration = 0
    matrix_.line_search_iteration = 0
    plant = make_plant(name)
    n = plant.get_num_pos()
    nx, nu = 2 * n, n
    cost = make_cost(nx, nu)
    x0, u0 = initial_problem(plant, N, dt, seed)
    solver = TrajoptMPCReference(plant, cost)
    m = {"S": SQPSolverMethods.S, "PCG-J": SQPSolverMethods.PCG_J, "PCG-BJ": SQPSolverMethods.PCG_BJ,
         "PCG-SS": SQPSolverMethods.PCG_SS, "N": SQPSolverMethods.N}[method]
    t0 = time.time()
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(copy.deepcopy(x0), copy.deepcopy(u0), N, dt, m, {})
    wall = time.time() - t0
    tr = solver.trace
    keys = ["iteration", "line_search_iteration", "alpha", "rho", "J", "c", "merit", "D", "reduction_ratio",
            "succeeded_line_search", "inner_iters", "singular"]
    rec = {"tr_" + k: np.array([np.nan if t[k] is None else float(t[k]) for t in tr]) for k in keys}
    pcg_iters = np.array([len(t[0][0]) - 1 for t in solver.saved_inner_traces], dtype=np.int32)
    # the |nu| trace of every QP's PCG (PCG.py:79-111), NaN-padded: where the exit test |nu'| < tol fell
    nu = np.full((len(pcg_iters), int(max(pcg_iters, default=0)) + 1), np.nan)
    for q, t in enumerate(solver.saved_inner_traces):
        nu[q, :len(t[0][0])] = np.asarray(t[0][0], dtype=float)
    dxul = np.array([d["value"][:, 0] for d in solver.saved_dxul])
    np.savez_compressed(os.path.join(OUT, f"sqp_{name}_N{N}_s{seed}_{method}.npz"),
                        x0=x0, u0=u0, x=np.asarray(x), u=np.asarray(u), dt=dt,
                        exit_sqp=exit_sqp, exit_soft=exit_soft, outer_iter=outer_iter, sqp_iter=sqp_iter,
                        pcg_iters=pcg_iters, nu_traces=nu, dxul=dxul, wall_s=wall, **rec)
    return f"[golden] sqp {name} N={N} seed={seed} {method}: exit={exit_sqp} iters={sqp_iter} " \
           f"pcg={list(pcg_iters)} wall={wall:.1f}s"


# ---------------------------------------------------------------- soft box constraints
def run_soft(args):
    """1-link arm, torque limits in a soft mode: the only box-constraint configuration the
    reference's TrajoptConstraint code runs (constraint_size 1).  Records the
    final trajectory, exit codes, the last outer iteration's trace and the final mu / lambda /
    phi of the torque BoxConstraint."""
    mode, method, N, q0, seed, dt = args
    _setup_reference()
    sys.path.insert(0, os.path.dirname(OUT))
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from trajoptmpcreference_amd.urdf import planar_arm_urdf
    from TrajoptPlant import URDFPlant
    from TrajoptConstraint import TrajoptConstraint
    from TrajoptMPCReference import TrajoptMPCReference, SQPSolverMethods
    from overloading import matrix_
    matrix_.iteration = 0
    matrix_.soft_constraint_iteration = 0
    matrix_.line_search_iteration = 0
    urdf = planar_arm_urdf(1)
    d = tempfile.mkdtemp(prefix="tmpc_urdf_")
    path = os.path.join(d, "arm1.urdf")
    with open(path, "w") as f:
        f.write(urdf)
    plant = URDFPlant(options={"path_to_urdf": path, "overloading": False})
    cost = make_cost(2, 1)
    rng = np.random.default_rng(seed)
    x0 = np.zeros((2, N))
    x0[0, 0] = q0 + rng.uniform(-0.1, 0.1)
    u0 = np.zeros((1, N - 1))
    for k in range(N - 1):
        x0[:, k + 1] = plant.integrator(x0[:, k], u0[:, k], dt)
    lb, ub = -0.5, 0.5
    con = TrajoptConstraint(1, 1, 1, N)
    con.overloading = False   # attribute the reference reads but never sets
    con.set_torque_limits([ub], [lb], mode, {"overloading": False})
    solver = TrajoptMPCReference(plant, cost, con)
    m = {"S": SQPSolverMethods.S, "PCG-BJ": SQPSolverMethods.PCG_BJ, "PCG-SS": SQPSolverMethods.PCG_SS}[method]
    import io
    import contextlib
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(copy.deepcopy(x0), copy.deepcopy(u0), N, dt, m,
                                                                     {"overloading": False})
    wall = time.time() - t0
    tr = solver.trace
    keys = ["outer_iteration", "iteration", "line_search_iteration", "alpha", "rho", "J", "c", "merit", "D",
            "reduction_ratio", "succeeded_line_search"]
    rec = {"tr_" + k: np.array([np.nan if t[k] is None else float(np.asarray(t[k]).reshape(-1)[0]) for t in tr])
           for k in keys}
    tl = con.torque_limits
    tag = {"QUADRATIC_PENALTY": "QP", "AUGMENTED_LAGRANGIAN": "AL"}[mode]
    np.savez_compressed(os.path.join(OUT, f"soft_arm1_N{N}_{tag}_s{seed}_{method}.npz"),
                        urdf=np.array(urdf), x0=x0, u0=u0, x=np.asarray(x), u=np.asarray(u), dt=dt, lb=lb, ub=ub,
                        mode=np.array(mode), exit_sqp=exit_sqp, exit_soft=exit_soft, outer_iter=outer_iter,
                        sqp_iter=sqp_iter, mu=tl.quadratic_penalty_mu, lam=tl.augmented_lagrangian_lambda,
                        phi=tl.augmented_lagrangian_phi, wall_s=wall, **rec)
    return f"[golden] soft {tag} {method} N={N} seed={seed}: exit_sqp={exit_sqp} exit_soft={exit_soft} " \
           f"outer={outer_iter} iters={sqp_iter} wall={wall:.1f}s"


def run_hard(args):
    """1-link arm, torque limits in a HARD mode (ACTIVE_SET / FULL_SET): the violated rows
    [u - lb; ub - u] < 0 are appended to C after each knot's dynamics rows
    (TrajoptMPCReference.py:238-248, TrajoptConstraint.py:53-130).  constraint_size 1 is the
    only size the reference's BoxConstraint runs.  Records, per QP, the active rows
    (knot, +1 lower / -1 upper) read back from the reference's own C, and the PCG counts."""
    mode, method, N, q0, seed, dt, erm = args
    _setup_reference()
    sys.path.insert(0, os.path.dirname(OUT))
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from trajoptmpcreference_amd.urdf import planar_arm_urdf
    from TrajoptPlant import URDFPlant
    from TrajoptConstraint import TrajoptConstraint
    from TrajoptMPCReference import TrajoptMPCReference, SQPSolverMethods
    from overloading import matrix_
    matrix_.iteration = 0
    matrix_.soft_constraint_iteration = 0
    matrix_.line_search_iteration = 0
    urdf = planar_arm_urdf(1)
    d = tempfile.mkdtemp(prefix="tmpc_urdf_")
    path = os.path.join(d, "arm1.urdf")
    with open(path, "w") as f:
        f.write(urdf)
    plant = URDFPlant(options={"path_to_urdf": path, "overloading": False})
    cost = make_cost(2, 1)
    rng = np.random.default_rng(seed)
    x0 = np.zeros((2, N))
    x0[0, 0] = q0 + rng.uniform(-0.1, 0.1)
    u0 = np.zeros((1, N - 1))
    for k in range(N - 1):
        x0[:, k + 1] = plant.integrator(x0[:, k], u0[:, k], dt)
    lb, ub = -0.5, 0.5
    con = TrajoptConstraint(1, 1, 1, N)
    con.overloading = False   # attribute the reference reads but never sets
    con.set_torque_limits([ub], [lb], mode, {"overloading": False})
    solver = TrajoptMPCReference(plant, cost, con)
    m = {"S": SQPSolverMethods.S, "PCG-J": SQPSolverMethods.PCG_J, "PCG-BJ": SQPSolverMethods.PCG_BJ,
         "PCG-SS": SQPSolverMethods.PCG_SS, "N": SQPSolverMethods.N}[method]
    opts = {"overloading": False}
    if erm is not None:
        opts["expected_reduction_min_SQP_DDP"] = erm
    import io
    import contextlib
    t0 = time.time()
    err = ""
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(copy.deepcopy(x0), copy.deepcopy(u0), N,
                                                                         dt, m, opts)
    except Exception as e:   # the reference's own failure, recorded as data
        err = repr(e)
        x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = x0, u0, -1, -1, -1, -1
    wall = time.time() - t0
    tr = solver.trace
    keys = ["iteration", "line_search_iteration", "alpha", "rho", "J", "c", "merit", "D", "reduction_ratio",
            "succeeded_line_search", "singular"]
    rec = {"tr_" + k: np.array([np.nan if t[k] is None else float(np.asarray(t[k]).reshape(-1)[0]) for t in tr])
           for k in keys}
    # active rows per QP from the reference's C: rows past nx*N, in order; knot = column block, sign = entry
    nx, n = 2, 3
    act_knot, act_sign, act_qp = [], [], []
    for q, dC in enumerate(solver.saved_C):
        C = np.asarray(dC["value"])
        for r in range(C.shape[0]):
            row = C[r]
            nzc = np.nonzero(row)[0]
            if r >= nx and len(nzc) == 1 and (nzc[0] % n) == nx:   # a torque row: one entry in a u column
                act_qp.append(q)
                act_knot.append(int(nzc[0] // n))
                act_sign.append(int(np.sign(row[nzc[0]])))
    pcg_iters = np.array([len(t[0][0]) - 1 for t in solver.saved_inner_traces], dtype=np.int32)
    dxul = [np.asarray(dd["value"])[:, 0] for dd in solver.saved_dxul]
    rows = np.array([np.asarray(dC["value"]).shape[0] for dC in solver.saved_C], dtype=np.int32)
    W = max([len(v) for v in dxul] + [1])
    dx_pad = np.array([np.concatenate([v, np.full(W - len(v), np.nan)]) for v in dxul]) if dxul else np.zeros((0, 1))
    tag = {"ACTIVE_SET": "AS", "FULL_SET": "FS"}[mode]
    np.savez_compressed(os.path.join(OUT, f"hard_arm1_N{N}_{tag}_s{seed}_{method}.npz"),
                        urdf=np.array(urdf), x0=x0, u0=u0, x=np.asarray(x), u=np.asarray(u), dt=dt, lb=lb, ub=ub,
                        mode=np.array(mode), erm=np.nan if erm is None else erm, error=np.array(err),
                        exit_sqp=exit_sqp, exit_soft=exit_soft, outer_iter=outer_iter, sqp_iter=sqp_iter,
                        pcg_iters=pcg_iters, C_rows=rows, act_qp=np.array(act_qp, dtype=np.int32),
                        act_knot=np.array(act_knot, dtype=np.int32), act_sign=np.array(act_sign, dtype=np.int32),
                        dxul=dx_pad, wall_s=wall, **rec)
    return f"[golden] hard {tag} {method} N={N} seed={seed} erm={erm}: exit_sqp={exit_sqp} iters={sqp_iter} " \
           f"rows={list(rows)} pcg={list(pcg_iters)} err={err[:80]} wall={wall:.1f}s"


def gen_soft_hooks(N=8, seed=2024):
    """The reference's soft-constraint plugin hooks on their own (TrajoptConstraint.py:53-166,
    295-378), 1-link arm (constraint_size 1, the size the reference's BoxConstraint runs):
    value_soft_constraints / jacobian_soft_constraints at random (x_k, u_k, k) with random mu /
    lambda / phi, and update_soft_constraint_constants on random trajectories (flag + constants after).
    Torque limits (N-1 knots) and joint limits (the reference sizes them N-1 knots, so the
    trajectories keep knot N-1 inside the bounds) in QUADRATIC_PENALTY and AUGMENTED_LAGRANGIAN."""
    _setup_reference()
    from TrajoptConstraint import TrajoptConstraint
    rng = np.random.default_rng(seed)
    out = {"N": N}
    for kind in ("torque", "joint"):
        for mode, tag in (("QUADRATIC_PENALTY", "QP"), ("AUGMENTED_LAGRANGIAN", "AL")):
            con = TrajoptConstraint(1, 1, 1, N)
            con.overloading = False   # attribute the reference reads but never sets
            getattr(con, f"set_{kind}_limits")([0.5], [-0.5], mode, {"overloading": False})
            box = getattr(con, f"{kind}_limits")
            T = box.num_timesteps
            box.quadratic_penalty_mu[:] = 10.0 ** rng.uniform(-2, 2, (2, T))
            box.augmented_lagrangian_lambda[:] = rng.uniform(-1, 1, (2, T))
            box.augmented_lagrangian_phi[:] = 10.0 ** rng.uniform(-3, 0, (2, T))
            pre = f"{kind}_{tag}_"
            out[pre + "mu0"] = box.quadratic_penalty_mu.copy()
            out[pre + "lam0"] = box.augmented_lagrangian_lambda.copy()
            out[pre + "phi0"] = box.augmented_lagrangian_phi.copy()
            P = 24
            xs = rng.uniform(-1.2, 1.2, (P, 2))
            us = rng.uniform(-1.2, 1.2, (P, 1))
            ks = rng.integers(0, N - 1, P)
            vals, jacs = [], []
            for i in range(P):
                vals.append(float(np.asarray(con.value_soft_constraints(xs[i], us[i], int(ks[i]))).reshape(-1)[0]))
                jacs.append(np.asarray(con.jacobian_soft_constraints(xs[i], us[i], int(ks[i])), dtype=float).reshape(-1))
            out[pre + "xk"], out[pre + "uk"], out[pre + "k"] = xs, us, ks.astype(np.int32)
            out[pre + "value"], out[pre + "jac"] = np.array(vals), np.array(jacs)
            # AL updates on two random trajectories (|z| up to 0.8: some violations near phi, some far)
            flags, mus, lams, phis, Xs, Us = [], [], [], [], [], []
            for r in range(2):
                X = rng.uniform(-0.8, 0.8, (2, N))
                X[:, N - 1] = rng.uniform(-0.4, 0.4, 2)
                U = rng.uniform(-0.8, 0.8, (1, N - 1))
                flags.append(bool(con.update_soft_constraint_constants(X, U)))
                mus.append(box.quadratic_penalty_mu.copy())
                lams.append(box.augmented_lagrangian_lambda.copy())
                phis.append(box.augmented_lagrangian_phi.copy())
                Xs.append(X)
                Us.append(U)
            out[pre + "upd_x"], out[pre + "upd_u"] = np.array(Xs), np.array(Us)
            out[pre + "upd_flag"] = np.array(flags)
            out[pre + "upd_mu"], out[pre + "upd_lam"], out[pre + "upd_phi"] = np.array(mus), np.array(lams), np.array(phis)
    np.savez_compressed(os.path.join(OUT, "hooks_soft_arm1.npz"), **out)
    print(f"[golden] soft hooks: {len(out)} arrays")


def gen_soft_hooks_multi(N=8, seed=2025):
    """The reference's hooks with three soft kinds at once (joint QUADRATIC_PENALTY, velocity and torque
    AUGMENTED_LAGRANGIAN), 1-link arm: value_soft_constraints (the kinds' sum; BoxConstraint reads
    xk[:1], i.e. q, for the velocity kind too), jacobian_soft_constraints (the kinds' columns vstacked),
    max_soft_constraint_value, and update_soft_constraint_constants (`flag and update(...)`: once a
    kind returns False the later kinds are not updated) -- for TrajoptConstraint.reference_hooks.
    Joint limits are sized N - 1 knots by the reference, so the trajectories keep knot N - 1 inside."""
    _setup_reference()
    from TrajoptConstraint import TrajoptConstraint
    rng = np.random.default_rng(seed)
    con = TrajoptConstraint(1, 1, 1, N)
    con.overloading = False
    con.set_joint_limits([0.5], [-0.5], "QUADRATIC_PENALTY", {"overloading": False})
    con.set_velocity_limits([0.4], [-0.4], "AUGMENTED_LAGRANGIAN", {"overloading": False})
    con.set_torque_limits([0.3], [-0.3], "AUGMENTED_LAGRANGIAN", {"overloading": False})
    out = {"N": N}
    for kind in ("joint", "velocity", "torque"):
        box = getattr(con, f"{kind}_limits")
        T = box.num_timesteps
        box.quadratic_penalty_mu[:] = 10.0 ** rng.uniform(-2, 2, (2, T))
        box.augmented_lagrangian_lambda[:] = rng.uniform(-1, 1, (2, T))
        box.augmented_lagrangian_phi[:] = 10.0 ** rng.uniform(-3, 0, (2, T))
        out[f"{kind}_mu0"] = box.quadratic_penalty_mu.copy()
        out[f"{kind}_lam0"] = box.augmented_lagrangian_lambda.copy()
        out[f"{kind}_phi0"] = box.augmented_lagrangian_phi.copy()
    P = 24
    xs = rng.uniform(-1.2, 1.2, (P, 2))
    us = rng.uniform(-1.2, 1.2, (P, 1))
    ks = rng.integers(0, N - 1, P)
    vals, jacs = [], []
    for i in range(P):
        vals.append(float(np.asarray(con.value_soft_constraints(xs[i], us[i], int(ks[i]))).reshape(-1)[0]))
        jacs.append(np.asarray(con.jacobian_soft_constraints(xs[i], us[i], int(ks[i])), dtype=float))
    out["xk"], out["uk"], out["k"] = xs, us, ks.astype(np.int32)
    out["value"], out["jac"] = np.array(vals), np.array(jacs)
    res = {f"upd_{kind}_{a}": [] for kind in ("joint", "velocity", "torque") for a in ("mu", "lam", "phi")}
    flags, maxv, Xs, Us = [], [], [], []
    for r in range(4):
        X = rng.uniform(-0.9, 0.9, (2, N))
        X[:, N - 1] = rng.uniform(-0.3, 0.3, 2)
        U = rng.uniform(-0.9, 0.9, (1, N - 1))
        maxv.append(float(con.max_soft_constraint_value(X, U)))
        flags.append(bool(con.update_soft_constraint_constants(X, U)))
        for kind in ("joint", "velocity", "torque"):
            box = getattr(con, f"{kind}_limits")
            res[f"upd_{kind}_mu"].append(box.quadratic_penalty_mu.copy())
            res[f"upd_{kind}_lam"].append(box.augmented_lagrangian_lambda.copy())
            res[f"upd_{kind}_phi"].append(box.augmented_lagrangian_phi.copy())
        Xs.append(X)
        Us.append(U)
    out["upd_x"], out["upd_u"], out["upd_flag"], out["max_value"] = np.array(Xs), np.array(Us), np.array(flags), np.array(maxv)
    out.update({k: np.array(v) for k, v in res.items()})
    np.savez_compressed(os.path.join(OUT, "hooks_soft_multi_arm1.npz"), **out)
    print(f"[golden] soft hooks, three kinds: flags {flags}")


def run_pendulum(args):
    """The pendulum of examples/pendulum.py on the reference's own URDFPlant / RBDReference: the
    reference imports a PendulumPlant it never defines, so the build's PendulumPlant is a
    URDF model (trajoptmpcreference_amd/urdf.py pendulum_urdf) and this runs that URDF through the
    reference: the example's cost, N = 20, torque limits +-7 in a hard mode, the example's options."""
    mode, method, N, lim = args
    _setup_reference()
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from trajoptmpcreference_amd.urdf import pendulum_urdf
    from TrajoptPlant import URDFPlant
    from TrajoptCost import QuadraticCost
    from TrajoptConstraint import TrajoptConstraint
    from TrajoptMPCReference import TrajoptMPCReference, SQPSolverMethods
    from overloading import matrix_
    matrix_.iteration = 0
    matrix_.soft_constraint_iteration = 0
    matrix_.line_search_iteration = 0
    urdf = pendulum_urdf()
    d = tempfile.mkdtemp(prefix="tmpc_urdf_")
    path = os.path.join(d, "pendulum.urdf")
    with open(path, "w") as f:
        f.write(urdf)
    plant = URDFPlant(options={"path_to_urdf": path, "overloading": False})

    class PassThroughQuadraticCost(QuadraticCost):
        def value(self, x, u=None, timestep=None, *a, **k):
            return QuadraticCost.value(self, x, u, timestep)

        def gradient(self, x, u=None, timestep=None, *a, **k):
            return QuadraticCost.gradient(self, x, u, timestep)

        def hessian(self, x, u=None, timestep=None, *a, **k):
            return QuadraticCost.hessian(self, x, u, timestep)

    xg = np.array([3.14159, 0.0])
    cost = PassThroughQuadraticCost(np.diag([1.0, 1.0]), np.diag([100.0, 100.0]), np.diag([0.1]), xg)
    con = TrajoptConstraint(1, 1, 1, N)
    con.overloading = False
    con.set_torque_limits([lim], [-lim], mode, {"overloading": False})
    solver = TrajoptMPCReference(plant, cost, con)
    m = {"S": SQPSolverMethods.S, "PCG-SS": SQPSolverMethods.PCG_SS, "PCG-BJ": SQPSolverMethods.PCG_BJ}[method]
    x0, u0 = np.zeros((2, N)), np.zeros((1, N - 1))
    opts = {"expected_reduction_min_SQP_DDP": -100, "overloading": False}
    import io
    import contextlib
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(copy.deepcopy(x0), copy.deepcopy(u0), N, 0.1, m,
                                                                     opts)
    wall = time.time() - t0
    tr = solver.trace
    keys = ["iteration", "line_search_iteration", "alpha", "rho", "J", "c", "merit", "D", "reduction_ratio",
            "succeeded_line_search"]
    rec = {"tr_" + k: np.array([np.nan if t[k] is None else float(np.asarray(t[k]).reshape(-1)[0]) for t in tr])
           for k in keys}
    pcg_iters = np.array([len(t[0][0]) - 1 for t in solver.saved_inner_traces], dtype=np.int32)
    rows = np.array([np.asarray(dC["value"]).shape[0] for dC in solver.saved_C], dtype=np.int32)
    # dynamics known answers on the same model
    rng = np.random.default_rng(5)
    X = np.column_stack([rng.uniform(-3, 3, 8), rng.uniform(-2, 2, 8)])
    U = rng.uniform(-5, 5, (8, 1))
    qdd = np.array([plant.forward_dynamics(X[i], U[i]) for i in range(8)]).reshape(8, -1)
    tag = {"ACTIVE_SET": "AS", "AUGMENTED_LAGRANGIAN": "AL"}[mode]
    np.savez_compressed(os.path.join(OUT, f"pendulum_N{N}_{tag}{int(lim)}_{method}.npz"),
                        urdf=np.array(urdf), x0=x0, u0=u0, x=np.asarray(x), u=np.asarray(u), xg=xg, lim=lim,
                        mode=np.array(mode), exit_sqp=exit_sqp, exit_soft=exit_soft, outer_iter=outer_iter,
                        sqp_iter=sqp_iter, pcg_iters=pcg_iters, C_rows=rows, X=X, U=U, qdd=qdd, wall_s=wall, **rec)
    return f"[golden] pendulum {tag}{lim} {method} N={N}: exit={exit_sqp} iters={sqp_iter} rows={list(rows)} " \
           f"pcg={list(pcg_iters)} wall={wall:.1f}s"


# ---------------------------------------------------------------- user plugins (the plugin-hook path)
def run_plugins(args):
    """The reference's SQP with two user plugins written against its own base classes
    (tests/plugin_models.py): CoupledCost (a TrajoptCost with an x-u cross term, time-varying) on arm3, and
    SpringPlant (a TrajoptPlant without URDF) with CoupledCost."""
    which, N, seed, method, dt = args
    _setup_reference()
    sys.path.insert(0, os.path.dirname(OUT))
    import plugin_models as pm
    from TrajoptMPCReference import TrajoptMPCReference, SQPSolverMethods
    from TrajoptCost import TrajoptCost
    from TrajoptPlant import TrajoptPlant
    from overloading import matrix_
    matrix_.iteration = 0
    matrix_.soft_constraint_iteration = 0
    matrix_.line_search_iteration = 0

    class CoupledCost(TrajoptCost):
        def __init__(self, nx, nu):
            self.arrs = pm.coupled_arrays(nx, nu)

        def value(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_value(x, u, timestep, self.arrs)

        def gradient(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_gradient(x, u, timestep, self.arrs)

        def hessian(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_hessian(x, u, timestep, self.arrs)

    class _Shim:
        overloading = False

    class SpringPlant(TrajoptPlant):
        def __init__(self):
            super().__init__(0, {"overloading": False})
            self.rbdReference = _Shim()

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

    if which == "cost":
        plant = make_plant("arm3")
        x0, u0 = initial_problem(plant, N, dt, seed)
    else:
        plant = SpringPlant()
        x0, u0 = pm.spring_initial(N, dt, seed)
    n = plant.get_num_pos()
    cost = CoupledCost(2 * n, n)
    solver = TrajoptMPCReference(plant, cost)
    m = {"S": SQPSolverMethods.S, "PCG-J": SQPSolverMethods.PCG_J, "PCG-BJ": SQPSolverMethods.PCG_BJ,
         "PCG-SS": SQPSolverMethods.PCG_SS, "N": SQPSolverMethods.N}[method]
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(copy.deepcopy(x0), copy.deepcopy(u0), N, dt, m, {})
    tr = solver.trace
    keys = ["iteration", "line_search_iteration", "alpha", "rho", "J", "c", "merit", "D", "reduction_ratio",
            "succeeded_line_search"]
    rec = {"tr_" + k: np.array([np.nan if t[k] is None else float(t[k]) for t in tr]) for k in keys}
    pcg_iters = np.array([len(t[0][0]) - 1 for t in solver.saved_inner_traces], dtype=np.int32)
    dxul = np.array([d["value"][:, 0] for d in solver.saved_dxul])
    np.savez_compressed(os.path.join(OUT, f"plugin_{which}_N{N}_s{seed}_{method}.npz"),
                        x0=x0, u0=u0, x=np.asarray(x), u=np.asarray(u), dt=dt, exit_sqp=exit_sqp,
                        exit_soft=exit_soft, outer_iter=outer_iter, sqp_iter=sqp_iter, pcg_iters=pcg_iters,
                        dxul=dxul, **rec)
    return f"[golden] plugin {which} N={N} seed={seed} {method}: exit={exit_sqp} iters={sqp_iter} " \
           f"pcg={list(pcg_iters)}"


def run_plugins_hard(args):
    """The reference's SQP with a user cost plugin (tests/plugin_models.py CoupledCost, written against the
    reference's TrajoptCost: an x-u cross term, time-varying) AND hard ACTIVE_SET torque limits on the
    1-link arm (constraint_size 1, the size the reference's BoxConstraint runs): the hard rows are
    appended to C after each knot's dynamics rows (TrajoptMPCReference.py:238-248) on the plugin's own
    blocks.  Records run_hard's fields (per-QP active rows from the reference's own C, PCG counts)."""
    method, N, q0, seed, dt = args
    _setup_reference()
    sys.path.insert(0, os.path.dirname(OUT))
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    import plugin_models as pm
    from trajoptmpcreference_amd.urdf import planar_arm_urdf
    from TrajoptPlant import URDFPlant
    from TrajoptCost import TrajoptCost
    from TrajoptConstraint import TrajoptConstraint
    from TrajoptMPCReference import TrajoptMPCReference, SQPSolverMethods
    from overloading import matrix_
    matrix_.iteration = 0
    matrix_.soft_constraint_iteration = 0
    matrix_.line_search_iteration = 0

    class CoupledCost(TrajoptCost):
        def __init__(self, nx, nu):
            self.arrs = pm.coupled_arrays(nx, nu)

        def value(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_value(x, u, timestep, self.arrs)

        def gradient(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_gradient(x, u, timestep, self.arrs)

        def hessian(self, x, u=None, timestep=None, *a, **k):
            return pm.coupled_hessian(x, u, timestep, self.arrs)

    urdf = planar_arm_urdf(1)
    d = tempfile.mkdtemp(prefix="tmpc_urdf_")
    path = os.path.join(d, "arm1.urdf")
    with open(path, "w") as f:
        f.write(urdf)
    plant = URDFPlant(options={"path_to_urdf": path, "overloading": False})
    rng = np.random.default_rng(seed)
    x0 = np.zeros((2, N))
    x0[0, 0] = q0 + rng.uniform(-0.1, 0.1)
    u0 = np.zeros((1, N - 1))
    for k in range(N - 1):
        x0[:, k + 1] = plant.integrator(x0[:, k], u0[:, k], dt)
    lb, ub = -0.2, 0.2
    con = TrajoptConstraint(1, 1, 1, N)
    con.overloading = False   # attribute the reference reads but never sets
    con.set_torque_limits([ub], [lb], "ACTIVE_SET", {"overloading": False})
    solver = TrajoptMPCReference(plant, CoupledCost(2, 1), con)
    m = {"S": SQPSolverMethods.S, "PCG-J": SQPSolverMethods.PCG_J, "PCG-BJ": SQPSolverMethods.PCG_BJ,
         "PCG-SS": SQPSolverMethods.PCG_SS, "N": SQPSolverMethods.N}[method]
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        x, u, exit_sqp, exit_soft, outer_iter, sqp_iter = solver.SQP(copy.deepcopy(x0), copy.deepcopy(u0), N, dt, m,
                                                                     {"overloading": False})
    tr = solver.trace
    keys = ["iteration", "line_search_iteration", "alpha", "rho", "J", "c", "merit", "D", "reduction_ratio",
            "succeeded_line_search", "singular"]
    rec = {"tr_" + k: np.array([np.nan if t[k] is None else float(np.asarray(t[k]).reshape(-1)[0]) for t in tr])
           for k in keys}
    nx, n = 2, 3
    act_knot, act_sign, act_qp = [], [], []
    for q, dC in enumerate(solver.saved_C):
        C = np.asarray(dC["value"])
        for r in range(C.shape[0]):
            row = C[r]
            nzc = np.nonzero(row)[0]
            if r >= nx and len(nzc) == 1 and (nzc[0] % n) == nx:   # a torque row: one entry in a u column
                act_qp.append(q)
                act_knot.append(int(nzc[0] // n))
                act_sign.append(int(np.sign(row[nzc[0]])))
    pcg_iters = np.array([len(t[0][0]) - 1 for t in solver.saved_inner_traces], dtype=np.int32)
    rows = np.array([np.asarray(dC["value"]).shape[0] for dC in solver.saved_C], dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, f"plugin_hard_arm1_N{N}_s{seed}_{method}.npz"),
                        urdf=np.array(urdf), x0=x0, u0=u0, x=np.asarray(x), u=np.asarray(u), dt=dt, lb=lb, ub=ub,
                        exit_sqp=exit_sqp, exit_soft=exit_soft, outer_iter=outer_iter, sqp_iter=sqp_iter,
                        pcg_iters=pcg_iters, C_rows=rows, act_qp=np.array(act_qp, dtype=np.int32),
                        act_knot=np.array(act_knot, dtype=np.int32), act_sign=np.array(act_sign, dtype=np.int32),
                        **rec)
    return f"[golden] plugin+hard {method} N={N} seed={seed}: exit_sqp={exit_sqp} iters={sqp_iter} rows={list(rows)} " \
           f"pcg={list(pcg_iters)}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="skip the slow arm6 N=64 solves")
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    _setup_reference()
    if a.only in (None, "dyn"):
        for name in ["arm2", "arm3", "arm6fix"]:
            gen_model_and_dynamics(name)
    if a.only in (None, "qp"):
        gen_qp("arm3", 32)
        gen_qp("arm6fix", 64)
        gen_qp("arm2", 8)
    if a.only in (None, "sqp"):
        jobs = [("arm2", 8, 0, "PCG-SS", 0.1), ("arm3", 8, 0, "PCG-SS", 0.1), ("arm3", 8, 1, "PCG-BJ", 0.1),
                ("arm3", 8, 2, "PCG-J", 0.1), ("arm3", 8, 3, "S", 0.1)]
        jobs += [("arm3", 32, s, "PCG-SS", 0.1) for s in range(4)]
        jobs += [("arm3", 32, 0, m, 0.1) for m in ["PCG-J", "PCG-BJ", "S"]]
        if not a.quick:
            jobs += [("arm6fix", 64, s, "PCG-SS", 0.1) for s in range(2)]
        # slow ones first so the pool drains evenly
        jobs.sort(key=lambda j: -j[1] * (2 if j[0].startswith("arm6") else 1))
        with mp.get_context("fork").Pool(min(8, len(jobs))) as pool:
            for msg in pool.imap_unordered(run_sqp, jobs):
                print(msg, flush=True)
    if a.only in (None, "ee"):
        gen_ee_points()
        gen_ee_recorded()
        jobs = [("d4", [-1.0, 1.5, 0.0, 0.0], "PCG-SS"), ("d3", [-1.18, -1.58, 0.0, 0.0], "PCG-SS"),
                ("d4", [-1.0, 1.5, 0.0, 0.0], "S")]
        with mp.get_context("fork").Pool(len(jobs)) as pool:
            for msg in pool.imap_unordered(run_ee_sqp, jobs):
                print(msg, flush=True)
    if a.only in (None, "hard"):
        jobs = [("ACTIVE_SET", "PCG-SS", 8, 2.0, 0, 0.1, None), ("ACTIVE_SET", "S", 8, 2.0, 1, 0.1, None),
                ("ACTIVE_SET", "PCG-BJ", 10, 1.5, 2, 0.1, None), ("ACTIVE_SET", "PCG-SS", 12, 2.5, 3, 0.1, -100.0),
                ("ACTIVE_SET", "PCG-J", 8, 2.0, 4, 0.1, None), ("FULL_SET", "PCG-SS", 8, 2.0, 5, 0.1, None),
                ("FULL_SET", "S", 8, 2.0, 6, 0.1, None), ("ACTIVE_SET", "PCG-BJ", 10, 2.5, 7, 0.1, None),
                ("ACTIVE_SET", "PCG-SS", 16, 2.2, 8, 0.1, None), ("ACTIVE_SET", "S", 12, 3.0, 9, 0.1, -100.0),
                # method N (the dense KKT solve): the active set's rows, and FULL_SET's singular KKT -> lstsq
                ("ACTIVE_SET", "N", 8, 2.0, 10, 0.1, None), ("FULL_SET", "N", 8, 2.0, 11, 0.1, None)]
        with mp.get_context("fork").Pool(min(8, len(jobs))) as pool:
            for msg in pool.imap_unordered(run_hard, jobs):
                print(msg, flush=True)
    if a.only in (None, "pendulum"):
        jobs = [("ACTIVE_SET", "S", 20, 7.0), ("ACTIVE_SET", "PCG-SS", 20, 7.0), ("ACTIVE_SET", "S", 20, 20.0),
                ("AUGMENTED_LAGRANGIAN", "S", 20, 7.0)]
        with mp.get_context("fork").Pool(len(jobs)) as pool:
            for msg in pool.imap_unordered(run_pendulum, jobs):
                print(msg, flush=True)
    if a.only == "sqpJ":   # the PCG-J solves again, now with their |nu| traces
        jobs = [("arm3", 8, 2, "PCG-J", 0.1), ("arm3", 32, 0, "PCG-J", 0.1)]
        with mp.get_context("fork").Pool(len(jobs)) as pool:
            for msg in pool.imap_unordered(run_sqp, jobs):
                print(msg, flush=True)
    if a.only in (None, "hooks"):
        gen_soft_hooks()
    if a.only in (None, "hooks_multi"):
        gen_soft_hooks_multi()
    if a.only in (None, "sqpN"):
        # method N (dense KKT, solveKKTSystem :313-359), the reference's default SQP method
        jobs = [("arm2", 8, 0, "N", 0.1), ("arm3", 8, 1, "N", 0.1), ("arm3", 32, 0, "N", 0.1)]
        with mp.get_context("fork").Pool(len(jobs)) as pool:
            for msg in pool.imap_unordered(run_sqp, jobs):
                print(msg, flush=True)
    if a.only in (None, "plugins"):
        jobs = [("cost", 10, 0, "PCG-SS", 0.1), ("cost", 10, 1, "N", 0.1), ("plant", 20, 0, "PCG-SS", 0.1),
                ("plant", 20, 1, "N", 0.1), ("plant", 20, 2, "PCG-BJ", 0.1)]
        with mp.get_context("fork").Pool(len(jobs)) as pool:
            for msg in pool.imap_unordered(run_plugins, jobs):
                print(msg, flush=True)
    if a.only in (None, "plugins_hard"):
        jobs = [("PCG-SS", 10, 2.0, 20, 0.1), ("S", 10, 2.0, 21, 0.1), ("N", 12, 2.5, 22, 0.1),
                ("PCG-BJ", 12, 2.2, 23, 0.1)]
        with mp.get_context("fork").Pool(len(jobs)) as pool:
            for msg in pool.imap_unordered(run_plugins_hard, jobs):
                print(msg, flush=True)
    if a.only in (None, "soft"):
        jobs = [("QUADRATIC_PENALTY", "PCG-SS", 8, 2.0, 0, 0.1), ("AUGMENTED_LAGRANGIAN", "PCG-SS", 8, 2.0, 0, 0.1),
                ("QUADRATIC_PENALTY", "S", 8, 2.0, 1, 0.1), ("AUGMENTED_LAGRANGIAN", "S", 8, 2.0, 1, 0.1),
                ("AUGMENTED_LAGRANGIAN", "PCG-BJ", 8, 1.5, 2, 0.1), ("QUADRATIC_PENALTY", "PCG-SS", 12, 2.5, 3, 0.1)]
        with mp.get_context("fork").Pool(min(8, len(jobs))) as pool:
            for msg in pool.imap_unordered(run_soft, jobs):
                print(msg, flush=True)


if __name__ == "__main__":
    main()
