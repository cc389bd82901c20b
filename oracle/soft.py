"""Soft box constraints (QUADRATIC_PENALTY / AUGMENTED_LAGRANGIAN) restated
from the reference, with vector semantics.  TEST INFRASTRUCTURE ONLY (see
oracle/__init__.py): used by tests/, smoke() and bench.py's cpu_baseline.

Reference: TrajoptConstraint.py BoxConstraint.value (:53-83), .jacobian
(:85-128), .max_soft_constraint_value (:130-135),
.update_soft_constraint_constants (:137-166); TrajoptConstraint.
value/jacobian_soft_constraints, max_soft_constraint_value,
update_soft_constraint_constants (:296-379); their use in
formKKTSystemBlocks (:220-225, :255-259), totalCost (:303-307), the line
search D (:633-646) and check_and_update_soft_constraints (:483-508).

Per box limit of one type (joint q, velocity qd, torque u; constraint_size cs)
and knot t, with z the limited slice of x_t or u_t:

    v = [z - lb; ub - z]                                   (2 cs)
    value  = sum_i mu_i v_i^2   (+ sum_i lam_i v_i  in AUGMENTED_LAGRANGIAN)
    jac    = sum_i (2 mu_i v_i (+ lam_i)) J_i,  J_i = +-e_{idx(i)} if v_i < 0 else 0

exactly the reference's arithmetic for cs = 1, the only size its code runs
(np.vstack of the two 1-D halves gives a (2, cs) array that the
(2cs x 2cs) `base` matmul rejects for cs > 1).  Deliberate, documented
corrections of the reference where it cannot run:
  * cs > 1: the same formulas elementwise over the 2 cs entries (F6);
  * joint limits cover all N knots (the reference sizes them N-1, then
    indexes knot N-1 in soft modes: IndexError);
  * at the terminal knot only the state part of a jacobian is used (the
    reference adds an n_xu column to an nx slice: shape error);
  * several soft limit types at once: the KKT gradient gets the SUM of the
    per-type jacobians and the Hessian block the sum of the per-type outer
    products (the reference vstacks the jacobians and fails); the AL update
    runs for every type (no short-circuit of `and`).
"""
import numpy as np

TYPES = ("joint", "velocity", "torque")
SOFT_MODES = ("QUADRATIC_PENALTY", "AUGMENTED_LAGRANGIAN")


def default_soft_options(options=None):
    """BoxConstraint.validate_constraint_mode defaults (TrajoptConstraint.py:38-46)."""
    o = {} if options is None else dict(options)
    o.setdefault("quadratic_penalty_mu_init", 1e-2)
    o.setdefault("quadratic_penalty_mu_factor", 10.0)
    o.setdefault("quadratic_penalty_mu_max", 1e12)
    o.setdefault("augmentated_lagrangian_phi_init", 1e-2)
    o.setdefault("augmentated_lagrangian_phi_factor", 10.0)
    return o


class SoftLimit:
    """One BoxConstraint in a soft mode over T knots."""

    def __init__(self, kind, n, N, lb, ub, mode, options=None):
        assert kind in TYPES and mode in SOFT_MODES
        self.kind, self.n, self.mode = kind, n, mode
        self.T = N - 1 if kind == "torque" else N
        self.lb = np.broadcast_to(np.asarray(lb, dtype=float), (n,)).copy()
        self.ub = np.broadcast_to(np.asarray(ub, dtype=float), (n,)).copy()
        self.o = default_soft_options(options)
        self.mu = self.o["quadratic_penalty_mu_init"] * np.ones((2 * n, self.T))
        self.lam = np.zeros((2 * n, self.T))
        self.phi = self.o["augmentated_lagrangian_phi_init"] * np.ones((2 * n, self.T))
        # column offset of the limited slice inside [x; u] (jacobian head columns, :190-206)
        self.off = {"joint": 0, "velocity": n, "torque": 2 * n}[kind]

    def slice(self, xk, uk):
        if self.kind == "joint":
            return xk[:self.n]
        if self.kind == "velocity":
            return xk[self.n:2 * self.n]
        return uk

    def full_value(self, z):
        return np.concatenate([z - self.lb, self.ub - z])

    def value(self, z, t):
        v = self.full_value(z)
        val = np.sum(self.mu[:, t].dot(np.square(v)))
        if self.mode == "AUGMENTED_LAGRANGIAN":
            val = val + self.lam[:, t] @ v
        return val

    def jacobian(self, z, t, width):
        """d value / d[x; u] restricted to `width` columns (n_xu, or nx at the terminal knot)."""
        v = self.full_value(z)
        n = self.n
        sign = np.concatenate([np.ones(n), -np.ones(n)]) * (v < 0)
        coef = 2 * self.mu[:, t] * v * sign
        if self.mode == "AUGMENTED_LAGRANGIAN":
            coef = coef + self.lam[:, t] * sign
        j = np.zeros(width)
        for i in range(2 * n):
            col = self.off + (i % n)
            if col < width and sign[i] != 0:
                j[col] += coef[i]
        return j

    def max_value(self, z_of_t):
        m = 0
        for t in range(self.T):
            m = max(m, abs(min(self.full_value(z_of_t(t)))))
        return m

    def update(self, z_of_t):
        flag = True
        for t in range(self.T):
            v = self.full_value(z_of_t(t))
            active = v < 0
            lflag = np.abs(v) < self.phi[:, t]
            for i in range(len(v)):
                if active[i] and not lflag[i]:
                    if self.mu[i, t] < self.o["quadratic_penalty_mu_max"]:
                        flag = False
                        self.mu[i, t] = min(self.o["quadratic_penalty_mu_max"],
                                            self.mu[i, t] * self.o["quadratic_penalty_mu_factor"])
                elif active[i] and lflag[i]:
                    flag = False
                    self.lam[i, t] += self.mu[i, t] * v[i]
                    self.phi[i, t] /= self.o["augmentated_lagrangian_phi_factor"]
        return flag


class SoftConstraints:
    """The soft part of TrajoptConstraint: joint, velocity, torque limits in that order."""

    def __init__(self, limits):
        self.limits = [l for l in limits if l is not None]

    def active_at(self, k, N):
        return [l for l in self.limits if k < l.T]

    def value(self, xk, uk, k, N):
        val = 0
        for l in self.active_at(k, N):
            val += l.value(l.slice(xk, uk), k)
        return val

    def jacobians(self, xk, uk, k, N, width):
        return [l.jacobian(l.slice(xk, uk), k, width) for l in self.active_at(k, N)]

    def max_value(self, x, u):
        m = 0
        for l in self.limits:
            m = max(m, l.max_value(lambda t, l=l: l.slice(x[:, t], u[:, t] if t < u.shape[1] else None)))
        return m

    def update(self, x, u):
        flag = True
        for l in self.limits:
            f = l.update(lambda t, l=l: l.slice(x[:, t], u[:, t] if t < u.shape[1] else None))
            flag = flag and f
        return flag
