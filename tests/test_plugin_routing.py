"""CPU: which plugins run on the device and which on the plugin-hook path (trajoptmpcreference_amd/hooks.py).

The reference's SQP calls whatever cost / plant / constraint hooks the caller's subclasses define
(TrajoptMPCReference.py:217-227, :296-310, :635-648; any TrajoptCost / TrajoptPlant subclass passes its
type check, :31-38).  The drop-in honours that: the built-in plugins -- and subclasses that override none of
their hooks -- run wholly on the device; a subclass overriding a hook, or any other TrajoptCost /
TrajoptPlant / TrajoptConstraint subclass, takes the plugin-hook path (the reference's loop over the
hooks, every QP on the GPU).  No override is ever silently ignored: the entry points without a hook path
(iLQR, MPC, the device QP) raise."""
import numpy as np
import pytest

from conftest import quad_cost_arrays


def _plant(n=3):
    from trajoptmpcreference_amd import URDFPlant, planar_arm_urdf
    return URDFPlant(options={"path_to_urdf": planar_arm_urdf(n)})


def _costs():
    from trajoptmpcreference_amd import QuadraticCost, TrajoptCost

    class Scaled(QuadraticCost):                      # overrides a hook: its answer differs
        def gradient(self, x, u=None, timestep=None, *a, **k):
            return 2.0 * QuadraticCost.gradient(self, x, u, timestep)

    class PassThrough(QuadraticCost):                 # the F4 adapter pattern: still the caller's hook
        def value(self, x, u=None, timestep=None, *a, **k):
            return QuadraticCost.value(self, x, u, timestep)

    class Tagged(QuadraticCost):                      # a subclass adding state only: device plugin
        label = "mine"

    class Own(TrajoptCost):
        def value(self, x, u=None, timestep=None, *a, **k):
            return 0.0

    return Scaled, PassThrough, Tagged, Own


def test_cost_routing():
    from trajoptmpcreference_amd import QuadraticCost, hooks
    Scaled, PassThrough, Tagged, Own = _costs()
    arrs = quad_cost_arrays(3)
    assert hooks.device_cost(QuadraticCost(*arrs)) is not None
    assert hooks.device_cost(Tagged(*arrs)) is not None
    assert hooks.device_cost(Scaled(*arrs)) is None
    assert hooks.device_cost(PassThrough(*arrs)) is None
    assert hooks.device_cost(Own()) is None
    assert hooks.overrides(Scaled(*arrs), QuadraticCost, hooks.COST_HOOKS) == ["gradient"]


def test_plant_routing():
    from trajoptmpcreference_amd import PendulumPlant, TrajoptPlant, URDFPlant, hooks, planar_arm_urdf

    class Damped(URDFPlant):
        def forward_dynamics(self, x, u, *a, **k):
            return URDFPlant.forward_dynamics(self, x, u) - 0.1 * np.asarray(x)[self.model.n:]

    class Named(PendulumPlant):
        pass

    class Own(TrajoptPlant):
        def get_num_pos(self):
            return 1

    assert hooks.device_plant(_plant())
    assert hooks.device_plant(PendulumPlant())
    assert hooks.device_plant(Named())
    assert not hooks.device_plant(Damped(options={"path_to_urdf": planar_arm_urdf(2)}))
    assert not hooks.device_plant(Own())


def test_constraint_routing():
    from trajoptmpcreference_amd import TrajoptConstraint, hooks

    class MyLimits(TrajoptConstraint):
        def value_soft_constraints(self, xk, uk=None, timestep=None):
            return 0.0

    assert hooks.device_constraints(TrajoptConstraint(3, 3, 3, 8))
    assert not hooks.device_constraints(MyLimits(3, 3, 3, 8))


def test_overriding_subclass_takes_the_hook_path(monkeypatch):
    """SQP with an overriding cost never reaches the device SQP (which would evaluate the built-in
    quadratic cost): it is routed to hooks.sqp_hooks_batch with the caller's object."""
    from trajoptmpcreference_amd import TrajoptMPCReference, hooks
    from trajoptmpcreference_amd import solver as solver_mod
    Scaled, _, _, _ = _costs()
    s = TrajoptMPCReference(_plant(), Scaled(*quad_cost_arrays(3)))
    seen = {}

    def fake(solver, ctx, x, u, N, dt, method, options):
        seen.update(cost=solver.cost, method=method, N=N)
        raise RuntimeError("routed")

    monkeypatch.setattr(hooks, "sqp_hooks_batch", fake)
    monkeypatch.setattr(solver_mod.TrajoptMPCReference, "_hook_context", lambda self, o: None)
    with pytest.raises(RuntimeError, match="routed"):
        s.SQP(np.zeros((6, 8)), np.zeros((3, 7)), 8, 0.1, "PCG-SS", {})
    assert seen == {"cost": s.cost, "method": "PCG-SS", "N": 8}


def test_entry_points_without_a_hook_path_raise():
    """iLQR / MPC have no plugin-hook path: an overriding cost raises instead of being ignored."""
    from trajoptmpcreference_amd import TrajoptMPCReference
    Scaled, _, _, _ = _costs()
    s = TrajoptMPCReference(_plant(), Scaled(*quad_cost_arrays(3)))
    with pytest.raises(NotImplementedError, match="caller's own"):
        s.iLQR(np.zeros((6, 8)), np.zeros((3, 7)), 8, 0.1, {})
    with pytest.raises(NotImplementedError, match="caller's own"):
        s.MPC(np.zeros((6, 8)), np.zeros((3, 7)), 8, 0.1, options={})


def test_hook_path_refuses_what_it_cannot_run():
    """Hard rows and long horizons take the banded plugin QP (tmpc_qp_blocks_banded_batch, GPU tests); what it
    cannot run is refused before any solve: FULL_SET with a PCG method (S singular, the reference's
    preconditioner raises), a hard row that is not a box row."""
    from trajoptmpcreference_amd import TrajoptConstraint, TrajoptMPCReference, hooks
    Scaled, _, _, _ = _costs()
    con = TrajoptConstraint(3, 3, 3, 8)
    con.set_torque_limits([1.0] * 3, [-1.0] * 3, "FULL_SET")
    s = TrajoptMPCReference(_plant(), Scaled(*quad_cost_arrays(3)), con)
    o = {}
    s.set_default_options(o)
    with pytest.raises(NotImplementedError, match="FULL_SET"):
        hooks.sqp_hooks_batch(s, None, np.zeros((1, 6, 8)), np.zeros((1, 3, 7)), 8, 0.1, "PCG-SS", o)

    class SkewRows(TrajoptConstraint):   # a hard row over two entries: not a box row
        def jacobian_hard_constraints(self, xk, uk=None, timestep=None):
            J = super().jacobian_hard_constraints(xk, uk, timestep)
            if J is not None:
                J = J.copy()
                J[:, 0] += 0.5
            return J

    con2 = SkewRows(3, 3, 3, 8)
    con2.set_torque_limits([0.1] * 3, [-0.1] * 3, "ACTIVE_SET")
    s2 = TrajoptMPCReference(_plant(), Scaled(*quad_cost_arrays(3)), con2)
    q = hooks._HookSQP(s2, None, 8, 0.1, "PCG-SS", o)
    u = np.full((3, 7), 0.5)   # every torque above its bound: active rows at every knot
    with pytest.raises(NotImplementedError, match="box row"):
        q.hard_rows(np.zeros((6, 8)), u)
