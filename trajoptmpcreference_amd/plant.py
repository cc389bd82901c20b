"""TrajoptPlant / URDFPlant -- the reference's plant plugin surface
(TrajoptPlant.py:10-331), evaluated on the GPU.

Hooks keep the reference signatures (including the unused iter_* tracing
arguments).  Every numeric call goes through libtmpc (one lane per knot);
the batched ``*_batch`` variants are the efficient entry points.  Only the
explicit Euler integrator (type 0) -- the one every configuration uses -- is
offered; the other integrator ids raise (they are unused and their
gradients are inconsistent in the reference, TrajoptPlant.py:189,193,235-243).
"""
import numpy as np

from . import _native
from ._options import NO_OPTIONS, fresh
from .urdf import parse_urdf, pendulum_urdf


class _RBDReferenceShim:
    """The one attribute SQP reads from plant.rbdReference (TrajoptMPCReference.py:97,124)."""
    overloading = False


class TrajoptPlant:
    """Base plant (TrajoptPlant.py:10-108)."""

    def __init__(self, integrator_type: int = 0, options=NO_OPTIONS, need_path: bool = False):
        self.validate_integrator_type(integrator_type)
        self.integrator_type = integrator_type
        options = fresh(options)
        self.set_default_options(options, need_path)
        self.options = options

    def validate_integrator_type(self, integrator_type: int):
        if integrator_type not in [0, 1, 2, 3, 4, -1]:
            raise ValueError("Invalid integrator options are [0 : euler, 1 : semi-implicit euler, 2 : midpoint, "
                             "3 : rk3, 4 : rk4, -1 : hard-coded as dynamics")
        if integrator_type != 0:
            raise NotImplementedError("only the explicit Euler integrator (type 0) runs on the GPU")

    def set_default_options(self, options: dict, need_path: bool = False):
        options.setdefault("path_to_urdf", None)
        options.setdefault("gravity", -9.81)
        options.setdefault("overloading", False)
        if need_path and not options.get("path_to_urdf"):
            raise ValueError("You must include the 'path_to_urdf' in the options.")

    def forward_dynamics(self, x, u, iter_1=0, iter_2=0, iter_3=0):
        raise NotImplementedError

    def forward_dynamics_gradient(self, x, u, iter_1=0, iter_2=0, iter_3=0):
        raise NotImplementedError

    def get_num_pos(self):
        raise NotImplementedError

    def get_num_vel(self):
        raise NotImplementedError

    def get_num_cntrl(self):
        raise NotImplementedError

    def qdd_to_xdot(self, xk, qdd):
        """[v; qdd] (TrajoptPlant.py:61-68)."""
        nq = self.get_num_pos()
        return np.concatenate((np.asarray(xk)[nq:], np.asarray(qdd)))

    def dqdd_to_dxdot(self, dqdd):
        """[[0, I, 0]; dqdd] (TrajoptPlant.py:72-81)."""
        nq, nv, m = self.get_num_pos(), self.get_num_vel(), self.get_num_cntrl()
        top = np.hstack((np.zeros((nq, nq)), np.eye(nv), np.zeros((nq, m))))
        return np.vstack((top, dqdd))

    def integrator(self, xk, uk, dt, return_gradient=False, iter_1=0, iter_2=0, iter_3=0):
        """TrajoptPlant.integrator, explicit Euler (TrajoptPlant.py:83-108) on this plant's own
        forward_dynamics / forward_dynamics_gradient hooks: x+ = x + dt [v; qdd], A = I + dt dxdot_x,
        B = dt dxdot_u.  URDFPlant overrides it with the GPU's batched kernels."""
        xk = np.asarray(xk, dtype=np.float64)
        n = len(xk)
        qdd = self.forward_dynamics(xk, uk, iter_1, iter_2, iter_3)
        xkp1 = xk + dt * self.qdd_to_xdot(xk, qdd)
        if not return_gradient:
            return xkp1
        dxdot = self.dqdd_to_dxdot(self.forward_dynamics_gradient(xk, uk, iter_1, iter_2, iter_3))
        return np.eye(n) + dt * dxdot[:, 0:n], dt * dxdot[:, n:]


class URDFPlant(TrajoptPlant):
    """URDF rigid-body plant (TrajoptPlant.py:274-331) on the GPU."""

    def __init__(self, integrator_type: int = 0, options=NO_OPTIONS, device: int = 0):
        options = fresh(options)
        super().__init__(integrator_type, options, True)
        path = options["path_to_urdf"]
        self.model = parse_urdf(path)
        self.robot = self.model
        self.rbdReference = _RBDReferenceShim()
        self.device = device

    # context with this plant's model loaded
    def _ctx(self):
        ctx = _native.default_context(self.device)
        if ctx.model is not self.model:
            ctx.set_model(self.model, self.options["gravity"])
        return ctx

    def get_num_pos(self):
        return self.model.n

    def get_num_vel(self):
        return self.model.n

    def get_num_cntrl(self):
        return self.model.n

    # -- batched entry points (K knots at once)
    def forward_dynamics_batch(self, x, u):
        _, qdd, _ = self._ctx().fd_batch(np.atleast_2d(x), np.atleast_2d(u), 0.0, want_minv=False)
        return qdd

    def minv_batch(self, q):
        q = np.atleast_2d(q)
        x = np.hstack((q, np.zeros_like(q)))
        _, _, Mi = self._ctx().fd_batch(x, np.zeros_like(q), 0.0, want_minv=True)
        return Mi

    def forward_dynamics_gradient_batch(self, x, u):
        _, _, dq = self._ctx().fd_grad_batch(np.atleast_2d(x), np.atleast_2d(u), 0.0)
        return dq

    def integrator_batch(self, x, u, dt, return_gradient=False):
        ctx = self._ctx()
        if not return_gradient:
            xn, _, _ = ctx.fd_batch(np.atleast_2d(x), np.atleast_2d(u), dt, want_minv=False)
            return xn
        A, B, _ = ctx.fd_grad_batch(np.atleast_2d(x), np.atleast_2d(u), dt)
        return A, B

    # -- reference hook signatures (single knot)
    def forward_dynamics(self, x, u, iter_1=0, iter_2=0, iter_3=0):
        return self.forward_dynamics_batch(np.asarray(x)[None], np.asarray(u)[None])[0]

    def forward_dynamics_gradient(self, x, u, iter_1=0, iter_2=0, iter_3=0):
        return self.forward_dynamics_gradient_batch(np.asarray(x)[None], np.asarray(u)[None])[0]

    def integrator(self, xk, uk, dt, return_gradient=False, iter_1=0, iter_2=0, iter_3=0):
        """Euler step / its Jacobians (TrajoptPlant.py:83-108)."""
        r = self.integrator_batch(np.asarray(xk)[None], np.asarray(uk)[None], dt, return_gradient)
        if return_gradient:
            return r[0][0], r[1][0]
        return r[0]


class PendulumPlant(URDFPlant):
    """The pendulum the reference's package and examples/pendulum.py import but TrajoptPlant.py never
    defines (__init__.py:1, examples/pendulum.py:7): one joint, nq = nv = nu = 1, a bob of
    `mass` at `length` below the pivot, so qdd = (u - m g l sin q) / (m l^2 + I_bob) and q = pi is
    upright (examples/pendulum.py's goal xg = [3.14159, 0]).  It is a URDF model (urdf.pendulum_urdf)
    behind the URDFPlant surface, so it runs on the same GPU kernels as every other plant."""

    def __init__(self, integrator_type: int = 0, options=NO_OPTIONS, device: int = 0, mass: float = 1.0,
                 length: float = 1.0):
        # a copy: the caller's dict must not come back pointing at the pendulum model
        options = dict(options)
        options["path_to_urdf"] = pendulum_urdf(mass, length)
        super().__init__(integrator_type, options, device)

