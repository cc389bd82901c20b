"""CPU restatement of the reference's end-effector cost `UrdfCost`
(TEST INFRASTRUCTURE: imported only by tests/, never by the product path).

Follows
  * TrajoptCost.py:371-569            UrdfCost value / gradient / hessian (hess_mode 0), get_currQ
  * GRiD/RBDReference/RBDReference.py:123-148   end_effector_positions
  * RBDReference.py:214-259           dJdq     (hand-coded 2-link formulas)
  * RBDReference.py:263-310           d2Jdq2   (hand-coded 2-link formulas)
  * RBDReference.py:313-331           jacobian_tot_state  d(x, y, vx, vy)/d(q, qd)
  * RBDReference.py:334-387           Jacobian (chain of H / dH, rows [:n, :n])

Task state y(x) = [p(q); J(q) qd] with p the first two coordinates of the leaf
position (offset [0, 1, 0, 1] in the leaf frame).  The reference hard-codes the
2-link Jacobian-derivative patterns, so like it this restatement is
defined for n = 2 only and raises otherwise.

Parity is pinned by tests/golden/ee_arm2*.npz (generated from the reference by
tests/golden/make_golden.py --ee) and by the recorded run
/root/reference/data/4/final_traj.csv / final_input.csv, copied
as data into tests/golden/ee_arm2_data4.npz.
"""
import numpy as np

OFFSET = np.array([0.0, 1.0, 0.0, 1.0])     # UrdfCost.offsets (TrajoptCost.py:388)


def _chain(model):
    """sorted(get_ancestors_by_id(leaf)) + [leaf] for the first leaf (RBDReference.py:137-139)."""
    children = {int(p) for p in model.parent if p >= 0}
    leaf = min(j for j in range(model.n) if j not in children)
    chain, j = [], leaf
    while j >= 0:
        chain.append(j)
        j = int(model.parent[j])
    return sorted(chain)


def _check(model):
    if model.n != 2 or model.H0 is None:
        raise ValueError("UrdfCost is defined for 2-link arms only (RBDReference.py:262-265,311-314; SURVEY F5)")


def end_effector_position(model, q):
    """end_effector_positions (RBDReference.py:123-148): (prod_i H_i(q_i)) @ offset, rows [:2]."""
    H = np.eye(4)
    for j in _chain(model):
        H = H @ model.H(j, q[j])
    return (H @ OFFSET)[:2]


def jacobian(model, q):
    """Jacobian (RBDReference.py:334-387): column d = chain with dH at joint d, rows [:n, :n]."""
    n = model.n
    chain = _chain(model)
    J = np.zeros((3, n))
    for d in range(n):
        if d not in chain:
            continue
        H = np.eye(4)
        for j in chain:
            H = H @ (model.dH(j, q[j]) if j == d else model.H(j, q[j]))
        J[:, d] = (H @ OFFSET)[:3]
    return J[:n, :n]


def dJdq(J):
    """RBDReference.py:252-259 (literal hand-coded pattern)."""
    return np.array([[-J[1, 0], -J[1, 1]],
                     [-J[1, 1], -J[1, 1]],
                     [-J[0, 0], -J[0, 1]],
                     [J[0, 1], J[0, 1]]])


def jacobian_tot_state(model, q, qd):
    """jacobian_tot_state (RBDReference.py:313-331): [[J, 0], [reshape(dJdq @ qd, (n, n)), J]]."""
    n = model.n
    J1 = jacobian(model, q)
    J2 = (dJdq(J1) @ qd).reshape(n, n)
    return np.vstack((np.hstack((J1, np.zeros_like(J1))), np.hstack((J2, J1))))


class UrdfCost:
    """UrdfCost (TrajoptCost.py:371-569), hess_mode 0 (Gauss-Newton, :490-492).
    Same hook shape as oracle.sqp.QuadCost, with the state-dependent hessian taking x."""

    state_hessian = True

    def __init__(self, model, Q, QF, R, xg, QF_start=None):
        _check(model)
        self.model = model
        self.n = model.n
        self.Q, self.QF, self.R, self.xg, self.QF_start = Q, QF, R, np.asarray(xg, dtype=float), QF_start

    def currQ(self, terminal, k):
        """get_currQ (:541-548)."""
        shifted = self.QF_start is not None and k is not None and k >= self.QF_start
        return self.QF if (terminal or shifted) else self.Q

    def delta_x(self, x):
        """delta_x (:425-435): [p(q); J(q) qd] - xg."""
        n = self.n
        q, qd = x[:n], x[n:]
        pos = end_effector_position(self.model, q)
        vel = jacobian(self.model, q) @ qd
        return np.concatenate((pos, vel)) - self.xg

    def value(self, x, u, k):
        """value (:402-422)."""
        dx = self.delta_x(x)
        v = 0.5 * (dx @ (self.currQ(u is None, k) @ dx))
        if u is not None:
            v += 0.5 * (u @ (self.R @ u))
        return v

    def gradient(self, x, u, k):
        """gradient (:437-458): [dx^T Q Jtot, u^T R]."""
        n = self.n
        dx = self.delta_x(x)
        Jt = jacobian_tot_state(self.model, x[:n], x[n:])
        top = (dx @ self.currQ(u is None, k)) @ Jt
        return top if u is None else np.hstack((top, u @ self.R))

    def hessian(self, u_is_none, k, x=None):
        """hessian, hess_mode 0 (:482-519): (Q Jtot)^T Jtot, blockdiag with R."""
        n = self.n
        Jt = jacobian_tot_state(self.model, x[:n], x[n:])
        hx = (self.currQ(u_is_none, k) @ Jt).T @ Jt
        if u_is_none:
            return hx
        nx, nu = hx.shape[0], self.R.shape[0]
        return np.vstack((np.hstack((hx, np.zeros((nx, nu)))), np.hstack((np.zeros((nu, nx)), self.R))))
