"""GPU parity past 1024 Schur rows: arm6 at N = 128 (1536 rows, BASELINE config 5)
on the SQP path.

Up to 1024 rows the fused QP kernel keeps every lane's rows of S and P^-1 in
registers; past that they no longer fit a CU's register file and the GM
instance keeps them in HBM (k_qp<..., GM>).  These tests check
that instance against
  * the oracle at N = 128 (tests/golden/oracle_arm6_N128_sqp_pcgss.npz and
    oracle_config5_arm6_N128_mpc_sqp_pcgss.npz, made by
    tests/golden/make_oracle_fixtures.py --only sqp128 / mpc128sqp), and
  * the reference's own recorded solves, by forcing the GM instance at
    N = 64 (TMPC_QP_GM_MIN_ROWS=1): exit codes, SQP / line-search iterations,
    per-QP PCG counts and alpha paths identical.
Integer outputs must be identical; trajectories within 1e-6 relative."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, arm_model, golden, quad_cost_arrays, replay_qp_counts

pytestmark = pytest.mark.gpu


def _solver(n):
    from trajoptmpcreference_amd import QuadraticCost, TrajoptMPCReference, URDFPlant, planar_arm_urdf
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})
    return TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(n)))


def _problems(N, seeds, dt=0.1):
    from oracle import sqp as osqp
    m = arm_model("arm6fix")
    xs, us = zip(*[osqp.initial_problem(m, N, dt, int(s)) for s in seeds])
    return np.array(xs), np.array(us)


def _rel(a, b):
    return float(np.max(np.abs(a - b))) / max(1.0, float(np.max(np.abs(b))))


def test_sqp_pcgss_arm6_n128_matches_oracle():
    d = golden("oracle_arm6_N128_sqp_pcgss.npz")
    N = int(d["N"])
    x, u = _problems(N, d["seeds"])
    r = _solver(6).SQP_batch(x, u, N, 0.1, "PCG-SS", {})
    for i in range(len(d["seeds"])):
        assert (int(r["exit_sqp"][i]), int(r["sqp_iter"][i])) == (int(d["exit_sqp"][i]), int(d["sqp_iter"][i])), i
        ref = [int(v) for v in d["pcg_iters"][i] if v >= 0]
        assert [int(v) for v in r["trace"]["pcg_iters"][i, 1:len(ref) + 1]] == ref, i
        al = d["alpha"][i]
        al = list(al[~np.isnan(al)])
        assert list(r["trace"]["alpha"][i, 1:len(al) + 1]) == al, i
        assert _rel(r["x"][i], d["x"][i]) < 1e-6, i
        assert _rel(r["u"][i], d["u"][i]) < 1e-6, i
    # integer parity on identical inputs: the GM instance against its canonical-order restatement
    solver = _solver(6)
    for i in range(2):
        nq = int(r["sqp_iter"][i]) + (1 if int(r["exit_sqp"][i]) == 3 else 0)
        counts = [int(v) for v in r["trace"]["pcg_iters"][i, 1:nq + 1]]
        ok = [bool(v) for v in r["trace"]["succeeded_line_search"][i, 1:nq + 1]]
        replay_qp_counts(solver, x[i:i + 1], u[i:i + 1], N, 0.1, "PCG-SS", counts, ok)


def test_sqp_pcgss_arm6_n128_warm_start_replay():
    """Config 5's QP path: the GM instance with the PCG warm start (each QP from the previous QP's
    lambda), every QP replayed exactly against the canonical order started from the same guess."""
    N = 128
    x, u = _problems(N, [975])
    solver = _solver(6)
    opts = {"pcg_warm_start": True}
    r = solver.SQP_batch(x, u, N, 0.1, "PCG-SS", dict(opts))
    nq = int(r["sqp_iter"][0]) + (1 if int(r["exit_sqp"][0]) == 3 else 0)
    assert nq >= 3
    counts = [int(v) for v in r["trace"]["pcg_iters"][0, 1:nq + 1]]
    ok = [bool(v) for v in r["trace"]["succeeded_line_search"][0, 1:nq + 1]]
    replay_qp_counts(solver, x, u, N, 0.1, "PCG-SS", counts, ok, opts=opts, warm=True)


def test_sqp_method_s_arm6_n128_matches_oracle():
    """Method S past 1024 rows: the GM instance's Schur prologue / dxu epilogue around k_btsolve."""
    from oracle import sqp as osqp
    m = arm_model("arm6fix")
    N = 128
    x, u = _problems(N, [970, 971])
    r = _solver(6).SQP_batch(x, u, N, 0.1, "S", {})
    for i in range(2):
        o = osqp.sqp(m, osqp.QuadCost(*quad_cost_arrays(6)), x[i], u[i], N, 0.1, "S")
        assert (int(r["exit_sqp"][i]), int(r["sqp_iter"][i])) == (o["exit_sqp"], o["sqp_iter"]), i
        assert _rel(r["x"][i], o["x"]) < 1e-6, i


def test_config5_mpc_loop_sqp_pcgss_arm6_n128():
    """BASELINE config 5 on SQP: the MPC loop with PCG-SS horizon solves and the PCG warm start."""
    d = golden("oracle_config5_arm6_N128_mpc_sqp_pcgss.npz")
    N, steps = int(d["N"]), int(d["steps"])
    x, u = _problems(N, d["seeds"])
    r = _solver(6).MPC_batch(x, u, N, 0.1, "QP-PCG-SS", {"pcg_warm_start": True}, mpc_steps=steps)
    for i in range(len(d["seeds"])):
        assert list(r["exit_codes"][i]) == list(d["exit_codes"][i]), i
        assert list(r["iters"][i]) == list(d["iters"][i]), i
        assert np.allclose(r["x_exec"][i], d["x_exec"][i], rtol=1e-6, atol=1e-8), i
        assert np.allclose(r["u_exec"][i], d["u_exec"][i], rtol=1e-6, atol=1e-8), i


# the GM instance's PCG-J counts where they differ from the reference's recorded ones (test_gpu_sqp.py
# PCGJ_ORDER_DECIDED): fixture -> {QP index: (the GPU's count, the reference's)}
PCGJ_ORDER_DECIDED_GM = {
    "sqp_arm3_N8_s2_PCG-J.npz": {1: (58, 59)},
}


@pytest.mark.parametrize("f", sorted(glob.glob(os.path.join(GOLDEN, "sqp_arm*_N*_s*_PCG-*.npz"))),
                         ids=lambda f: os.path.basename(f))
def test_gm_instance_matches_reference_fixtures(f, monkeypatch):
    """The HBM-row instance forced at the reference's own sizes (N <= 64) reproduces its solves."""
    monkeypatch.setenv("TMPC_QP_GM_MIN_ROWS", "1")
    b = os.path.basename(f)[4:-4]
    name, Ns, _, method = b.split("_")
    N = int(Ns[1:])
    from conftest import ARM_N
    d = np.load(f)
    solver = _solver(ARM_N[name])
    x, u, exit_sqp, _, _, sqp_iter = solver.SQP(d["x0"], d["u0"], N, float(d["dt"]), method, {})
    assert (exit_sqp, sqp_iter) == (int(d["exit_sqp"]), int(d["sqp_iter"]))
    tr = solver.trace
    assert [t["alpha"] for t in tr] == list(d["tr_alpha"])
    ours = [t["inner_iters"] for t in tr[1:]]
    if method == "PCG-J":   # test_gpu_sqp.py: the QPs whose Jacobi CG count the rounding of S decides
        from test_gpu_sqp import pcgj_diffs
        assert ours[0] == int(d["pcg_iters"][0])
        assert pcgj_diffs(ours, d["pcg_iters"]) == PCGJ_ORDER_DECIDED_GM.get(os.path.basename(f), {})
    else:
        assert ours == list(d["pcg_iters"])
    replay_qp_counts(solver, d["x0"][None], d["u0"][None], N, float(d["dt"]), method, ours,
                     [t["succeeded_line_search"] for t in tr[1:]], gm_min_rows=1)
    rtol = 1e-4 if method == "PCG-J" else 1e-7
    assert _rel(x, d["x"]) < rtol
    assert _rel(u, d["u"]) < rtol


BIG = sorted(glob.glob(os.path.join(GOLDEN, "oracle_big_*.npz")))


@pytest.mark.parametrize("f", BIG, ids=lambda f: os.path.basename(f))
def test_sqp_past_the_fused_rows_matches_oracle(f):
    """Past the fused QP's 1536 Schur rows the QP takes the banded path of the hard-limit kernels with no
    constraint rows (csrc/tmpc_api.cpp qp_banded): a 7-joint chain at N = 128 (1792 rows, PCG-SS) and arm6 at
    N = 256 (3072 rows, method S: the banded direct elimination), against the oracle in that path's canonical
    order (tests/golden/oracle_big_*.npz, make_oracle_fixtures.py --only big): exit code, SQP iterations, the
    alpha path and every PCG count identical, trajectories within 1e-6; and every QP of the GPU's own run
    replayed at its own iterate -- the canonical-order PCG (oracle/hard.py pcg_canonical) on the QP's own
    banded S takes the GPU's count and returns its lambda bit for bit (test_gpu_hard._replay_pcg_counts)."""
    from oracle import hard as ohard
    from oracle import sqp as osqp
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    from test_gpu_hard import _replay_pcg_counts
    d = np.load(f)
    n = int(os.path.basename(f).split("_")[2][3:])
    N, method = int(d["N"]), os.path.basename(f)[:-4].split("_")[-1]
    m = parse_urdf(planar_arm_urdf(n))
    x0, u0 = osqp.initial_problem(m, N, 0.1, int(d["seed"]))
    x, u = x0[None], u0[None]
    solver = _solver(n)
    tol = float(d["exit_tolerance_linSys"]) if "exit_tolerance_linSys" in d else float("nan")
    opts = {} if np.isnan(tol) else {"exit_tolerance_linSys": tol}
    r = solver.SQP_batch(x, u, N, 0.1, method, dict(opts), hard_active=True)
    got = (int(r["exit_sqp"][0]), int(r["sqp_iter"][0]))
    assert got == (int(d["exit_sqp"]), int(d["sqp_iter"])), got
    nq = got[1] + (1 if got[0] == 3 else 0)
    assert list(r["trace"]["alpha"][0, 1:nq + 1]) == list(d["alpha"])
    if method.startswith("PCG"):
        assert [int(v) for v in r["trace"]["pcg_iters"][0, 1:nq + 1]] == [int(v) for v in d["pcg_iters"]]
    assert _rel(r["x"][0], d["x"]) < 1e-6
    assert _rel(r["u"][0], d["u"]) < 1e-6
    if method.startswith("PCG"):
        _replay_pcg_counts(solver, r, x, u, N, method, ohard.HardConstraints([]), n, base_opts=opts)


def test_banded_path_refuses_warm_start():
    """The banded PCG takes no guess: pcg_warm_start past the fused rows is an error, not ignored."""
    from trajoptmpcreference_amd import _native
    x, u = _problems(130, [5])
    with pytest.raises(_native.NativeError, match="warm"):
        _solver(6).SQP_batch(x, u, 130, 0.1, "PCG-SS", {"pcg_warm_start": True})


def test_banded_path_refuses_a_horizon_past_the_schur_kernels_lds():
    """The banded Schur kernel (k_hard_schur) keeps per-knot and per-row records in LDS: past 160 KB a
    horizon is refused with the largest supported N named (arm6 without hard limits: N = 650), before any
    launch -- not a generic launch failure."""
    from trajoptmpcreference_amd import _native
    N = 651
    x, u = _problems(N, [3])
    with pytest.raises(_native.NativeError, match="largest supported horizon .* is N = 650"):
        _solver(6).SQP_batch(x, u, N, 0.1, "S", {"max_iter_SQP_DDP": 1})
