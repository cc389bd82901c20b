"""GPU parity of the bench's hard-limit workload itself: arm6 (joint 6 fixed), N = 64, SQP PCG-SS, ACTIVE_SET
torque +-0.5 and velocity +-1 limits on every joint (bench.py LIMIT_PRESETS "torque-velocity-as";
TrajoptMPCReference.py:238-248, 609-744), 8 problems of the bench workload (seeds 0..7) against the oracle's
SQP in the banded PCG's canonical summation order (tests/golden/oracle_hard_arm6_N64_torque_velocity_as.npz,
tests/golden/make_oracle_fixtures.py --only hard6).

Per problem (one test each):
  * identical runs: exit code, SQP iterations, every QP's PCG count, the alpha path, the line-search outcomes,
    every QP's per-knot active-set bitmasks and singular flag -- all exact;
  * a run that parts from the oracle's (most QPs of this workload stop at the 100-iteration PCG cap, so the
    runs' directions differ by what the last bits of their S amplify to, and a problem whose line-search
    trial sits at the acceptance threshold can take the other step) must be explained by the replay of
    bench.classify_hard_mismatch at the first point the runs part, or the test fails: every integer before
    that point identical; at the GPU's own iterate the oracle's line search along the GPU's direction takes
    the GPU's outcome and along the oracle's own direction (its dense KKT solve at that iterate, canonical
    order) a different one -- the decision sits where the two directions' rounding-amplified difference
    flips it ("line_search"; on such a problem the oracle's own runs on two hosts differ too: its dense KKT
    formation goes through the host's BLAS); or the canonical PCG on the GPU's own S takes the GPU's count
    ("pcg_count");
  * every QP of the GPU's own run is replayed at the GPU's own iterate (test_gpu_hard._replay_pcg_counts):
    tmpc_qp_batch takes the trace's PCG count and active set, and the canonical-order PCG on that QP's S
    reproduces the count and the GPU's lambda bit for bit."""
import numpy as np
import pytest

from conftest import arm_model, golden, quad_cost_arrays

pytestmark = pytest.mark.gpu

FIXTURE = "oracle_hard_arm6_N64_torque_velocity_as.npz"


def _solver(N, d):
    from trajoptmpcreference_amd import (QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant,
                                         planar_arm_urdf)
    plant = URDFPlant(options={"path_to_urdf": planar_arm_urdf(6)})
    con = TrajoptConstraint(6, 6, 6, N)
    con.set_torque_limits([float(d["ub_u"])] * 6, [float(d["lb_u"])] * 6, "ACTIVE_SET")
    con.set_velocity_limits([float(d["ub_v"])] * 6, [float(d["lb_v"])] * 6, "ACTIVE_SET")
    return TrajoptMPCReference(plant, QuadraticCost(*quad_cost_arrays(6)), con)


@pytest.mark.parametrize("i", range(8))
def test_hard_arm6_n64_problem_matches_oracle(i):
    import bench
    from oracle import hard as ohard
    from oracle import sqp as osqp
    from test_gpu_hard import _replay_pcg_counts
    d = golden(FIXTURE)
    N = int(d["N"])
    solver = _solver(N, d)
    x0, u0 = osqp.initial_problem(arm_model("arm6fix"), N, 0.1, int(d["seeds"][i]))
    x0, u0 = x0[None], u0[None]
    r = solver.SQP_batch(x0, u0, N, 0.1, "PCG-SS", {}, hard_active=True)
    ex, it = int(r["exit_sqp"][0]), int(r["sqp_iter"][0])
    nq = it + (1 if ex == 3 else 0)
    tr = r["trace"]
    got = dict(counts=[int(v) for v in tr["pcg_iters"][0, 1:nq + 1]],
               alpha=[float(v) for v in tr["alpha"][0, 1:nq + 1]],
               succ=[bool(v) for v in tr["succeeded_line_search"][0, 1:nq + 1]],
               masks=[[int(v) for v in tr["hard_active"][0, q + 1]] for q in range(nq)],
               sing=[bool(v) for v in tr["singular"][0, 1:nq + 1]])
    rq = int(d["sqp_iter"][i]) + (1 if int(d["exit_sqp"][i]) == 3 else 0)
    ref = dict(counts=[int(v) for v in d["pcg_iters"][i] if v >= 0],
               alpha=[float(v) for v in d["alpha"][i, :rq]], succ=[bool(v) for v in d["succeeded"][i, :rq]],
               masks=[[int(v) for v in d["masks"][i, q]] for q in range(rq)],
               sing=[bool(v) for v in d["singular"][i, :rq]])
    same = (ex, it) == (int(d["exit_sqp"][i]), int(d["sqp_iter"][i])) and got == ref
    if same:
        scale = max(1.0, float(np.max(np.abs(d["x"][i]))))
        assert float(np.max(np.abs(r["x"][0] - d["x"][i]))) < 1e-6 * scale
    else:
        opts = {}
        solver.set_default_options(opts)
        ctx = solver._context(opts)
        why = bench.classify_hard_mismatch(ctx, x0, u0, N, 0.1, "PCG-SS", r, 0,
                                           dict(pcg_iters=ref["counts"], alpha=ref["alpha"], succeeded=ref["succ"]),
                                           "torque-velocity-as")
        import warnings
        warnings.warn(f"hard arm6 problem {i} (seed {int(d['seeds'][i])}) parts from the oracle: {why}")
        assert why["kind"] is not None, why
        j = why["j"]
        # every decision before the parting point identical, and the QPs up to it saw the same active sets
        assert got["counts"][:j] == ref["counts"][:j] and got["alpha"][:j] == ref["alpha"][:j], (j, got, ref)
        assert got["succ"][:j] == ref["succ"][:j] and got["sing"][:j + 1] == ref["sing"][:j + 1], j
        assert got["masks"][:j + 1] == ref["masks"][:j + 1], j
    hard = ohard.HardConstraints([ohard.HardLimit("torque", 6, float(d["lb_u"]), float(d["ub_u"]), "ACTIVE_SET"),
                                  ohard.HardLimit("velocity", 6, float(d["lb_v"]), float(d["ub_v"]), "ACTIVE_SET")])
    _replay_pcg_counts(solver, r, x0, u0, N, "PCG-SS", hard, 6)
