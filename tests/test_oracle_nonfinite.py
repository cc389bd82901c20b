"""CPU: the oracle's treatment of diverging line-search trials.

A trial whose rollout overflows gives J_new = inf or NaN; the acceptance test of
the reference (TrajoptMPCReference.py:659-666 for SQP, the same ratio window in
oracle/ilqr.py) is `ratio >= min and ratio <= max`, false for a NaN ratio and
for +-inf, so the trial is rejected and alpha halves.  These tests pin that the
oracle actually meets such trials on the iLQR workload the GPU tests use
(test_gpu_ilqr.py::test_ilqr_nonfinite_trials_rejected compares the GPU on
exactly these problems) and that rejection leaves a finite solution.
"""
import numpy as np

from conftest import arm_model, quad_cost_arrays


def test_ratio_window_rejects_nonfinite():
    from oracle import sqp as osqp
    o = osqp.default_options({})
    lo, hi = o["expected_reduction_min_SQP_DDP"], o["expected_reduction_max_SQP_DDP"]
    for ratio in (np.float64("nan"), np.float64("inf"), np.float64("-inf")):
        assert not (ratio >= lo and ratio <= hi)


def test_ilqr_diverging_trials_are_rejected(monkeypatch):
    from oracle import ilqr as oilqr
    from oracle import sqp as osqp
    m = arm_model("arm3")
    N = 32
    seen = []
    fwd = oilqr.forward

    def forward(*a, **k):
        xn, un = fwd(*a, **k)
        seen.append(bool(np.all(np.isfinite(xn)) and np.all(np.isfinite(un))))
        return xn, un

    monkeypatch.setattr(oilqr, "forward", forward)
    cost = osqp.QuadCost(*quad_cost_arrays(3))
    x, u = osqp.initial_problem(m, N, 0.1, 502)   # problem 2 of the GPU test's batch
    with np.errstate(over="ignore", invalid="ignore"):
        o = oilqr.ilqr(m, cost, x, u, N, 0.1, {})
    assert not all(seen), "seed 502 no longer produces a diverging trial"
    assert np.all(np.isfinite(o["x"])) and np.all(np.isfinite(o["u"]))
    assert all(np.isfinite(t["J"]) for t in o["trace"])
    # every accepted step has a finite ratio inside the window
    acc = [t for t in o["trace"][1:] if t["succeeded_line_search"]]
    assert acc and all(np.isfinite(t["reduction_ratio"]) for t in acc)
