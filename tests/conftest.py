import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")

ARM_N = {"arm2": 2, "arm3": 3, "arm6fix": 6, "arm7": 7}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libtmpc.so")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


def arm_model(name):
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    return parse_urdf(planar_arm_urdf(ARM_N[name]))


def quad_cost_arrays(n):
    nx = 2 * n
    return np.eye(nx), 100.0 * np.eye(nx), 0.1 * np.eye(n), np.zeros(nx)


@pytest.fixture(scope="session")
def ctx():
    from trajoptmpcreference_amd import _native
    return _native.default_context(0)


def replay_qp_counts(solver, x0, u0, N, dt, method, counts, succeeded, opts=None, gm_min_rows=None, warm=False):
    """Integer parity of every QP of one GPU SQP run without a tolerance: QP j is replayed at the GPU's
    own iterate (the same solve stopped after j iterations, rho_j from the trace's schedule,
    check_for_exit_or_error TrajoptMPCReference.py:463-481) through tmpc_qp_batch, which must take the
    trace's PCG count, and the canonical-order PCG (oracle/canon.c, in the lane layout the kernel ran:
    one row of S per lane, or two -- past 768 rows and in the HBM-row GM instance, which
    TMPC_QP_GM_MIN_ROWS = gm_min_rows forces) on that QP's own S and gamma must take it too and return
    the GPU's lambda bit for bit (solveKKTSystem_Schur :415-445 + PCG.py:66-111 on identical inputs).
    warm: the PCG warm start (options 'pcg_warm_start'; PCG.py:11-12, TrajoptMPCReference.py:439-440):
    QP j starts from QP j - 1's lambda, QP 0 from zeros.  x0 / u0 [1][nx][N] / [1][nu][N-1].
    Returns the lambdas."""
    from oracle import canon
    base = dict(opts or {})
    o = dict(base)
    solver.set_default_options(o)
    f = float(o["rho_factor_SQP_DDP"])
    rho, drho = o["rho_init_SQP_DDP"], 1.0
    nx = x0.shape[1]
    prev = np.zeros(N * nx) if warm else None
    lams = []
    for j, want in enumerate(counts):
        if j == 0:
            xj, uj = x0, u0
        else:
            rj = solver.SQP_batch(x0, u0, N, dt, method, dict(base, max_iter_SQP_DDP=j))
            xj, uj = rj["x"], rj["u"]
        ctx = solver._context(dict(o))
        q = ctx.qp_batch(xj, uj, N, dt, rho, method, want_blocks=True, xs=x0[:, :, 0],
                         guess=None if prev is None else prev[None])
        assert int(q["pcg_iters"][0]) == want, (j, int(q["pcg_iters"][0]), want)
        lam, it, _ = canon.pcg(q["S_diag"][0], q["S_lo"][0], q["gamma"][0], method[4:],
                               tol=o["exit_tolerance_linSys"], max_iter=o["max_iter_linSys"],
                               rpl=canon.qp_rpl(N, nx, gm_min_rows), guess=prev)
        assert it == want, (j, it, want)
        assert np.array_equal(lam, q["dxul"][0][-N * nx:]), j
        lams.append(lam)
        if warm:
            prev = lam
        drho = min(drho / f, 1.0 / f) if succeeded[j] else max(drho * f, f)
        rho = max(rho * drho, o["rho_min_SQP_DDP"])
    return lams


def derived_exit(trace, opts):
    """(exit_sqp, sqp_iter) as check_for_exit_or_error (TrajoptMPCReference.py:463-481) derives them from a
    run's own trace rows (one per QP after the initial row): a failed line search raises rho and exits 2
    past rho_max; an accepted step exits 1 when J decreased by less than the tolerance (signed); the last
    allowed iteration exits 3."""
    o = dict(opts)
    f, rho, drho = float(o["rho_factor_SQP_DDP"]), o["rho_init_SQP_DDP"], 1.0
    J = trace[0]["J"]
    for it, t in enumerate(trace[1:]):
        ex = 0
        if t["succeeded_line_search"]:
            drho = min(drho / f, 1.0 / f)
            rho = max(rho * drho, o["rho_min_SQP_DDP"])
            if J - t["J"] < o["exit_tolerance_SQP_DDP"]:
                ex = 1
            J = t["J"]
        else:
            drho = max(drho * f, f)
            rho = max(rho * drho, o["rho_min_SQP_DDP"])
            if rho > o["rho_max_SQP_DDP"]:
                ex = 2
        if it == o["max_iter_SQP_DDP"] - 1:
            return 3, it
        if ex:
            return ex, it + 1
    return 0, len(trace) - 1
