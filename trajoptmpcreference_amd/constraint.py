"""TrajoptConstraint / BoxConstraint -- the reference's constraint plugin
surface (TrajoptConstraint.py:5-387).

Soft modes (QUADRATIC_PENALTY, AUGMENTED_LAGRANGIAN) run on the GPU: the
solver lowers the limits to ``tmpc_set_box_limits`` and the objects' mu /
lambda / phi arrays to ``tmpc_set_soft_state``, and stores the updated
constants back after the solve, as the reference's SQP updates them in place
(TrajoptMPCReference.py:483-508, TrajoptConstraint.py:137-166).

Semantics are the reference's for constraint_size 1 (the only size its code
runs) and the elementwise vector generalisation for larger sizes,
with the corrections documented in oracle/soft.py: joint limits cover all N
knots, terminal jacobians keep the state part, several soft types sum their
jacobians (and their per-type outer products in the KKT Hessian).

The hard modes (ACTIVE_SET / FULL_SET) append rows to C / c per knot
(TrajoptMPCReference.py:238-248); the GPU builds the resulting variable-size,
banded Schur complement per problem and reproduces the reference's nx-aligned
PCG preconditioner on it (csrc/tmpc_hard.hip).  Their semantics are the
reference's for constraint_size 1 and the elementwise generalisation above
(oracle/hard.py).  FULL_SET leaves zero rows in C for the inactive entries; the
reference's PCG then raises LinAlgError and its method S falls back to lstsq, so
FULL_SET runs with method S only.

The host-side value / jacobian / update methods below are the reference's plugin
hooks (value/jacobian_hard_constraints, value/jacobian_soft_constraints,
update/shift_soft_constraint_constants, ...) for callers that evaluate constraints
themselves; the GPU solve computes the same quantities on the device and never
calls them.
"""
from typing import List

import numpy as np

from ._options import NO_OPTIONS, fresh

HARD_MODES = ("ACTIVE_SET", "FULL_SET")
SOFT_MODES = ("QUADRATIC_PENALTY", "AUGMENTED_LAGRANGIAN", "ADMM_PROJECTION")
GPU_SOFT_MODES = ("QUADRATIC_PENALTY", "AUGMENTED_LAGRANGIAN")


class BoxConstraint:
    """lb <= z <= ub on a constraint_size slice (TrajoptConstraint.py:5-176)."""

    def __init__(self, constraint_size: int = 0, num_timesteps: int = 0, upper_bounds: List[float] = (),
                 lower_bounds: List[float] = (), mode: str = "NONE", options=NO_OPTIONS):
        options = fresh(options)
        self.constraint_size = constraint_size
        self.num_timesteps = num_timesteps
        self.num_constraints = 2 * constraint_size * num_timesteps
        lblen, ublen = len(lower_bounds), len(upper_bounds)
        if (lblen != constraint_size and lblen != 1) or (ublen != constraint_size and ublen != 1):
            raise ValueError("please enter bounds of the size of constraint or constant 1")
        self.bounds = np.zeros(2 * constraint_size)
        self.bounds[:constraint_size] = lower_bounds
        self.bounds[constraint_size:] = upper_bounds
        self.validate_constraint_mode(mode, options)
        T, m = num_timesteps, 2 * constraint_size
        self.quadratic_penalty_mu = options["quadratic_penalty_mu_init"] * np.ones((m, T))
        self.augmented_lagrangian_lambda = np.zeros((m, T))
        self.augmented_lagrangian_phi = options["augmentated_lagrangian_phi_init"] * np.ones((m, T))

    def validate_constraint_mode(self, mode: str, options=NO_OPTIONS):
        """TrajoptConstraint.py:37-51: set the mode and the option defaults (raises where the reference
        prints + exits)."""
        options = fresh(options)
        if mode not in HARD_MODES + SOFT_MODES:
            raise ValueError("Invalid Constraint Mode. Options are [ACTIVE_SET, FULL_SET, QUADRATIC_PENALTY, "
                             "AUGMENTED_LAGRANGIAN, ADMM_PROJECTION]")
        self.mode = mode
        options.setdefault("quadratic_penalty_mu_init", 1e-2)
        options.setdefault("quadratic_penalty_mu_factor", 10.0)
        options.setdefault("quadratic_penalty_mu_max", 1e12)
        options.setdefault("augmentated_lagrangian_phi_init", 1e-2)
        options.setdefault("augmentated_lagrangian_phi_factor", 10.0)
        options.setdefault("jacobian_extra_columns_head", 0)
        options.setdefault("jacobian_extra_columns_tail", 0)
        self.options = options

    def is_hard_constraint_mode(self, mode=None):
        return (self.mode if mode is None else mode) in HARD_MODES

    def is_soft_constraint_mode(self, mode=None):
        return (self.mode if mode is None else mode) in SOFT_MODES

    @property
    def lower(self):
        return self.bounds[:self.constraint_size]

    @property
    def upper(self):
        return self.bounds[self.constraint_size:]

    # ---- plugin API on the host (BoxConstraint.value / jacobian / ..., :53-176)
    def full_value(self, z):
        z = np.asarray(z, dtype=np.float64).reshape(-1)[:self.constraint_size]
        return np.concatenate([z - self.lower, self.upper - z])

    def value(self, xk, timestep: int = None, mode: str = None):
        mode = self.mode if mode is None else mode
        v = self.full_value(xk)
        if mode == "ACTIVE_SET":
            return v[v < 0]
        if mode == "FULL_SET":
            return v
        if mode in GPU_SOFT_MODES:
            if timestep is None:
                raise ValueError("Need Timestep for Soft Constraint Mode")
            val = np.sum(self.quadratic_penalty_mu[:, timestep].dot(np.square(v)))
            if mode == "AUGMENTED_LAGRANGIAN":
                val = val + self.augmented_lagrangian_lambda[:, timestep] @ v
            return val
        raise NotImplementedError("ADMM_PROJECTION is not implemented (the reference exits too, :81-83)")

    def jacobian(self, xk, timestep: int = None, mode: str = None):
        """Soft modes: the jacobian column (head + constraint_size + tail entries)."""
        mode = self.mode if mode is None else mode
        v = self.full_value(xk)
        cs = self.constraint_size
        sign = np.concatenate([np.ones(cs), -np.ones(cs)]) * (v < 0)
        full = np.zeros((2 * cs, cs))
        for i in range(2 * cs):
            full[i, i % cs] = sign[i]
        head, tail = self.options["jacobian_extra_columns_head"], self.options["jacobian_extra_columns_tail"]
        full = np.hstack([np.zeros((2 * cs, head)), full, np.zeros((2 * cs, tail))])
        if mode == "ACTIVE_SET":
            return full[~np.all(full == 0, axis=1)]
        if mode == "FULL_SET":
            return full
        if timestep is None:
            raise ValueError("Need Timestep for Soft Constraint Mode")
        jac = 2 * np.matmul(self.quadratic_penalty_mu[:, timestep] * v, full)
        if mode == "AUGMENTED_LAGRANGIAN":
            jac = jac + np.matmul(self.augmented_lagrangian_lambda[:, timestep], full)
        return jac.reshape(-1, 1)

    def max_soft_constraint_value(self, x):
        """TrajoptConstraint.py:131-136 on the limited slice x (constraint_size x num_timesteps)."""
        m = 0
        for t in range(self.num_timesteps):
            m = max(m, abs(min(self.full_value(x[:, t]))))
        return m

    def update_soft_constraint_constants(self, x):
        """BoxConstraint.update_soft_constraint_constants (:138-166) on the limited slice z_of_t
        (constraint_size x num_timesteps, one column per knot): per entry of [z - lb; ub - z] < 0,
        mu *= mu_factor (capped at mu_max) when |value| >= phi, else lambda += mu value and
        phi /= phi_factor.  Returns True when no constant changed (every violated mu at its cap)."""
        z_of_t = np.asarray(x, dtype=np.float64)
        o = self.options
        flag = True
        for t in range(self.num_timesteps):
            v = self.full_value(z_of_t[:, t])
            lflag = np.abs(v) < self.augmented_lagrangian_phi[:, t]
            for i in range(len(v)):
                if not v[i] < 0:
                    continue
                if not lflag[i]:
                    cur = self.quadratic_penalty_mu[i, t]
                    if cur < o["quadratic_penalty_mu_max"]:
                        flag = False
                        self.quadratic_penalty_mu[i, t] = min(o["quadratic_penalty_mu_max"],
                                                              cur * o["quadratic_penalty_mu_factor"])
                else:
                    flag = False
                    self.augmented_lagrangian_lambda[i, t] += self.quadratic_penalty_mu[i, t] * v[i]
                    self.augmented_lagrangian_phi[i, t] /= o["augmentated_lagrangian_phi_factor"]
        return flag

    def shift_soft_constraint_constants(self, shift_steps: int):
        """Receding-horizon shift (:168-176)."""
        for arr, init in ((self.quadratic_penalty_mu, self.options["quadratic_penalty_mu_init"]),
                          (self.augmented_lagrangian_lambda, 0.0),
                          (self.augmented_lagrangian_phi, self.options["augmentated_lagrangian_phi_init"])):
            arr[:, :-shift_steps] = arr[:, shift_steps:]
            arr[:, shift_steps:] = init


class TrajoptConstraint:
    """Joint / velocity / torque limits (TrajoptConstraint.py:178-387).

    The host hooks have two semantics.  By default (``reference_hooks = False``) they are the device's:
    velocity limits act on the qd slice of x, several soft kinds sum their jacobian columns, and
    update_soft_constraint_constants updates every kind (oracle/soft.py, what the GPU solve computes).
    With ``reference_hooks = True`` they are the reference's, for callers that swap these hooks in for
    its own: every state kind reads x[:constraint_size] (q, also for velocity limits), the kinds'
    jacobian columns are vstacked, and the update is ``flag = flag and update(...)``, so once a kind
    returns False the later kinds are left as they are (TrajoptConstraint.py:295-378; pinned bit for
    bit to the reference's own evaluation, tests/test_plugin_hooks.py)."""

    KINDS = ("joint_limits", "velocity_limits", "torque_limits")
    reference_hooks = False

    def __init__(self, nq: int = 0, nv: int = 0, nu: int = 0, num_timesteps: int = 0):
        self.nq, self.nv, self.nu, self.num_timesteps = nq, nv, nu, num_timesteps
        self.joint_limits = None
        self.velocity_limits = None
        self.torque_limits = None

    def set_joint_limits(self, upper_bounds, lower_bounds, mode, options=NO_OPTIONS):
        options = dict(options)
        options["jacobian_extra_columns_tail"] = self.nv + self.nu
        # all N knots (the reference sizes joint limits N-1 and then indexes knot N-1: oracle/soft.py)
        self.joint_limits = BoxConstraint(self.nq, self.num_timesteps, upper_bounds, lower_bounds, mode, options)

    def set_velocity_limits(self, upper_bounds, lower_bounds, mode, options=NO_OPTIONS):
        options = dict(options)
        options["jacobian_extra_columns_head"] = self.nq
        options["jacobian_extra_columns_tail"] = self.nu
        self.velocity_limits = BoxConstraint(self.nv, self.num_timesteps, upper_bounds, lower_bounds, mode, options)

    def set_torque_limits(self, upper_bounds, lower_bounds, mode, options=NO_OPTIONS):
        options = dict(options)
        options["jacobian_extra_columns_head"] = self.nq + self.nv
        self.torque_limits = BoxConstraint(self.nu, self.num_timesteps - 1, upper_bounds, lower_bounds, mode, options)

    def limits(self):
        return [(k, getattr(self, k)) for k in self.KINDS if getattr(self, k) is not None]

    def has_any(self) -> bool:
        return bool(self.limits())

    def total_soft_constraints(self, timestep=None):
        total = 0
        for kind, c in self.limits():
            if c.is_soft_constraint_mode():
                if timestep is None:
                    total += c.num_constraints
                elif not (kind == "torque_limits" and timestep >= self.num_timesteps - 1):
                    total += c.constraint_size
        return total

    def _hard_slices(self, xk, uk, timestep):
        """(kind, constraint, z) of the hard limits at a knot, in value_hard_constraints' order
        (:210-240); torque limits have no terminal-knot rows (:230)."""
        T = self.num_timesteps
        t = T - 1 if timestep is None else timestep
        out = []
        for kind, c in self.limits():
            if not c.is_hard_constraint_mode():
                continue
            if kind == "torque_limits":
                if t >= T - 1 or uk is None:
                    continue
                z = np.asarray(uk, dtype=np.float64).reshape(-1)
            elif kind == "joint_limits":
                z = np.asarray(xk, dtype=np.float64).reshape(-1)[:self.nq]
            else:
                z = np.asarray(xk, dtype=np.float64).reshape(-1)[self.nq:self.nq + self.nv]
            out.append((kind, c, z))
        return out

    def value_hard_constraints(self, xk, uk=None, timestep=None):
        """TrajoptConstraint.value_hard_constraints (:210-240), stacked 1-D."""
        vals = [c.value(z) for _, c, z in self._hard_slices(xk, uk, timestep)]
        return np.concatenate(vals) if vals else None

    def jacobian_hard_constraints(self, xk, uk=None, timestep=None):
        """TrajoptConstraint.jacobian_hard_constraints (:242-274): rows over [q; qd; u] (terminal: the
        state columns)."""
        n_xu = self.nq + self.nv + self.nu
        rows = []
        for kind, c, z in self._hard_slices(xk, uk, timestep):
            v = c.full_value(z)
            cs = c.constraint_size
            col0 = {"joint_limits": 0, "velocity_limits": self.nq, "torque_limits": self.nq + self.nv}[kind]
            for e in range(2 * cs):
                active = v[e] < 0
                if c.mode == "ACTIVE_SET" and not active:
                    continue
                r = np.zeros(n_xu)
                if active:
                    r[col0 + e % cs] = 1.0 if e < cs else -1.0
                rows.append(r)
        if not rows:
            return None
        J = np.array(rows)
        T = self.num_timesteps
        return J[:, :self.nq + self.nv] if (timestep is not None and timestep >= T - 1) else J

    def len_or_none(self, x):
        """TrajoptConstraint.py:276-279."""
        return 0 if x is None else len(x)

    def total_hard_constraints(self, x, u, timestep=None):
        """TrajoptConstraint.total_hard_constraints (:281-293)."""
        if not any(c.is_hard_constraint_mode() for _, c in self.limits()):
            return 0
        T = self.num_timesteps
        x = np.asarray(x)
        ks = range(T) if timestep is None else [timestep]
        tot = 0
        for k in ks:
            v = self.value_hard_constraints(x[:, k], None if (k >= T - 1 or u is None) else np.asarray(u)[:, k], k)
            tot += 0 if v is None else len(v)
        return tot

    def _soft_slices(self, xk, uk, timestep):
        """(kind, constraint, z) of the soft limits at a knot in the reference's order (joint, velocity,
        torque; torque limits have no terminal-knot term, :305,327)."""
        T = self.num_timesteps
        t = T - 1 if timestep is None else timestep
        out = []
        for kind, c in self.limits():
            if not c.is_soft_constraint_mode():
                continue
            if kind == "torque_limits":
                if t >= T - 1 or uk is None:
                    continue
                z = np.asarray(uk, dtype=np.float64).reshape(-1)
            elif kind == "joint_limits" or self.reference_hooks:
                z = np.asarray(xk, dtype=np.float64).reshape(-1)[:self.nq]
            else:
                z = np.asarray(xk, dtype=np.float64).reshape(-1)[self.nq:self.nq + self.nv]
            out.append((kind, c, z, t))
        return out

    def value_soft_constraints(self, xk, uk=None, timestep=None):
        """TrajoptConstraint.value_soft_constraints (:295-307): the sum over the soft limits of
        sum_i mu_i v_i^2 (+ sum_i lambda_i v_i for AUGMENTED_LAGRANGIAN) at `timestep`
        (default: the terminal knot).  0 when no limit is soft.  Velocity limits act on the qd slice
        of xk (the reference's BoxConstraint reads xk[:constraint_size], i.e. q, for every kind:
        oracle/soft.py)."""
        val = 0
        for _, c, z, t in self._soft_slices(xk, uk, timestep):
            val = val + c.value(z, t)
        return val

    def jacobian_soft_constraints(self, xk, uk=None, timestep=None):
        """TrajoptConstraint.jacobian_soft_constraints (:309-337): the (nq + nv + nu) x 1 column
        d value_soft_constraints / d[x; u] at `timestep`, None when no limit is soft.  With several
        soft limit kinds the reference vstacks their columns (which its SQP cannot consume);
        here they are summed, the gradient of the summed value (oracle/soft.py)."""
        jac = None
        for _, c, z, t in self._soft_slices(xk, uk, timestep):
            j = c.jacobian(z, t)
            jac = j if jac is None else (np.vstack((jac, j)) if self.reference_hooks else jac + j)
        return jac

    def soft_outer(self, xk, uk=None, timestep=None):
        """The soft limits' term of the QP's Hessian block at `timestep`: formKKTSystemBlocks adds
        outer(jac, jac) of the jacobian column (:220-225, :255-259); with several soft kinds (whose columns
        the reference vstacks and cannot consume) it is the sum of the per-kind outer products,
        the term the device QP and oracle/soft.py form.  None when no limit is soft."""
        if self.reference_hooks:
            raise NotImplementedError("soft_outer: with reference_hooks the jacobians are vstacked (the "
                                      "reference's form, which no QP consumes)")
        H = None
        for _, c, z, t in self._soft_slices(xk, uk, timestep):
            j = np.asarray(c.jacobian(z, t), dtype=np.float64).reshape(-1)
            H = np.outer(j, j) if H is None else H + np.outer(j, j)
        return H

    def update_soft_constraint_constants(self, x, u):
        """TrajoptConstraint.update_soft_constraint_constants (:369-378) for trajectories x
        (nq + nv) x N and u nu x (N - 1): the AL update of every limit; True when no constant changed.
        Every limit is updated (the reference's `flag and update(...)` skips the later kinds once a
        flag is False, which would leave their constants stale: oracle/soft.py)."""
        x = np.asarray(x, dtype=np.float64)
        flag = True
        for kind, c in self.limits():
            if kind == "joint_limits" or (kind == "velocity_limits" and self.reference_hooks):
                z = x[:self.nq]
            elif kind == "velocity_limits":
                z = x[self.nq:self.nq + self.nv]
            else:
                z = np.asarray(u, dtype=np.float64)
            if self.reference_hooks:
                flag = flag and c.update_soft_constraint_constants(z)   # the reference's short circuit
            else:
                f = c.update_soft_constraint_constants(z)
                flag = flag and f
        return flag

    def max_soft_constraint_value(self, x, u):
        m = 0
        for kind, c in self.limits():
            if not c.is_soft_constraint_mode():
                continue
            if kind == "joint_limits":
                m = max(m, c.max_soft_constraint_value(np.asarray(x)[:self.nq]))
            elif kind == "velocity_limits":
                lo = 0 if self.reference_hooks else self.nq
                m = max(m, c.max_soft_constraint_value(np.asarray(x)[lo:lo + self.nv]))
            else:
                m = max(m, c.max_soft_constraint_value(np.asarray(u)))
        return m

    def shift_soft_constraint_constants(self, shift_steps: int):
        for _, c in self.limits():
            c.shift_soft_constraint_constants(shift_steps)

    # ---- lowering to libtmpc
    def gpu_spec(self):
        """{joint|velocity|torque: {mode, lb, ub, options}} for Context.set_box_limits."""
        spec = {}
        for kind, c in self.limits():
            if c.mode not in GPU_SOFT_MODES + HARD_MODES:
                raise NotImplementedError(f"constraint mode {c.mode} is not implemented (the reference exits)")
            if c.constraint_size != self.nq:
                raise ValueError(f"{kind}: constraint_size {c.constraint_size} != n = {self.nq}")
            spec[kind.split("_")[0]] = dict(mode=c.mode, lb=c.lower.copy(), ub=c.upper.copy(), options=c.options)
        return spec

    def pack_state(self, N):
        """The objects' (2n, T) mu / lambda / phi as one problem's [N][6n] soft state."""
        n = self.nq
        out = []
        for attr, fill in (("quadratic_penalty_mu", 1e-2), ("augmented_lagrangian_lambda", 0.0),
                           ("augmented_lagrangian_phi", 1e-2)):
            a = np.zeros((N, 6 * n))
            for t, kind in enumerate(self.KINDS):
                c = getattr(self, kind)
                if c is None:
                    a[:, t * 2 * n:(t + 1) * 2 * n] = fill
                    continue
                arr = getattr(c, attr)
                T = arr.shape[1]
                a[:T, t * 2 * n:(t + 1) * 2 * n] = arr.T
                if T < N:
                    a[T:, t * 2 * n:(t + 1) * 2 * n] = arr[:, -1:].T if T else fill
            out.append(a)
        return out

    def unpack_state(self, mu, lam, phi):
        """Store one problem's [N][6n] soft state back into the objects."""
        n = self.nq
        for t, kind in enumerate(self.KINDS):
            c = getattr(self, kind)
            if c is None or not c.is_soft_constraint_mode():
                continue
            T = c.num_timesteps
            c.quadratic_penalty_mu[:] = mu[:T, t * 2 * n:(t + 1) * 2 * n].T
            c.augmented_lagrangian_lambda[:] = lam[:T, t * 2 * n:(t + 1) * 2 * n].T
            c.augmented_lagrangian_phi[:] = phi[:T, t * 2 * n:(t + 1) * 2 * n].T
