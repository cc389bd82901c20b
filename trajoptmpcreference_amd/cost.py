"""TrajoptCost / QuadraticCost -- the reference's cost plugin surface
(TrajoptCost.py:12-104).

The hooks accept (and ignore) the iter_* tracing arguments that SQP passes,
which the reference's own QuadraticCost rejects.  The GPU solver
reads Q, QF, R, xg and QF_start and evaluates the cost on the device; these
host methods exist for the plugin contract and for callers that evaluate
costs themselves (e.g. examples/exampleHelpers.py:101-111).
"""
import numpy as np


class TrajoptCost:
    def value(self, *args, **kwargs):
        raise NotImplementedError

    def gradient(self, *args, **kwargs):
        raise NotImplementedError

    def hessian(self, *args, **kwargs):
        raise NotImplementedError


class QuadraticCost(TrajoptCost):
    """0.5 dx^T Q dx + 0.5 u^T R u with QF at the terminal knot / from QF_start."""

    def __init__(self, Q_in, QF_in, R_in, xg_in, QF_start=None):
        self.Q = np.array(Q_in, dtype=np.float64)
        self.QF = np.array(QF_in, dtype=np.float64)
        self.R = np.array(R_in, dtype=np.float64)
        self.xg = np.array(xg_in, dtype=np.float64)
        self.increaseCount_Q = 0
        self.increaseCount_QF = 0
        self.QF_start = QF_start

    def get_currQ(self, u=None, timestep=None):
        """TrajoptCost.py:40-47."""
        last_state = u is None
        shifted_QF = timestep is not None and self.QF_start is not None and timestep >= self.QF_start
        return self.QF if (last_state or shifted_QF) else self.Q

    def value(self, x, u=None, timestep=None, iter_1=0, iter_2=0, iter_3=0):
        delta_x = np.asarray(x) - self.xg
        currQ = self.get_currQ(u, timestep)
        cost = 0.5 * np.matmul(delta_x.transpose(), np.matmul(currQ, delta_x))
        if u is not None:
            u = np.asarray(u)
            cost += 0.5 * np.matmul(u.transpose(), np.matmul(self.R, u))
        return cost

    def gradient(self, x, u=None, timestep=None, iter_1=0, iter_2=0, iter_3=0):
        delta_x = np.asarray(x) - self.xg
        top = np.matmul(delta_x.transpose(), self.get_currQ(u, timestep))
        if u is None:
            return top
        return np.hstack((top, np.matmul(np.asarray(u).transpose(), self.R)))

    def hessian(self, x, u=None, timestep=None, iter_1=0, iter_2=0, iter_3=0):
        nx, nu = self.Q.shape[0], self.R.shape[0]
        currQ = self.get_currQ(u, timestep)
        if u is None:
            return currQ
        return np.vstack((np.hstack((currQ, np.zeros((nx, nu)))), np.hstack((np.zeros((nu, nx)), self.R))))

    # receding-horizon hooks (TrajoptCost.py:85-104)
    def increase_QF(self, multiplier: float = 2.0):
        self.QF *= multiplier
        self.increaseCount_QF += 1
        return self.increaseCount_QF

    def increase_Q(self, multiplier: float = 2.0):
        self.Q *= multiplier
        self.increaseCount_Q += 1
        return self.increaseCount_Q

    def reset_increase_count_QF(self):
        self.increaseCount_QF = 0

    def reset_increase_count_Q(self):
        self.increaseCount_Q = 0

    def shift_QF_start(self, shift: float = -1.0):
        self.QF_start += shift
        self.QF_start = max(self.QF_start, 0)
        return self.QF_start


class UrdfCost(QuadraticCost):
    """End-effector cost (TrajoptCost.py:371-569): the quadratic form acts on the
    task state y = [p(q); J(q) qd] of the leaf's offset point [0, 1, 0, 1]
    (RBDReference.py:123-148, 313-387) instead of on x.  Hessian: hess_mode 0,
    (Q Jt)^T Jt (:490-492).  Like the reference it is defined for
    2-link arms only.  The GPU solver evaluates it on the device (ee_eval in
    csrc/tmpc_device.h); these host hooks serve callers that evaluate costs
    themselves."""

    OFFSET = np.array([0.0, 1.0, 0.0, 1.0])

    def __init__(self, plant, Q_in, QF_in, R_in, xg_in, QF_start=None, overloading=False):
        super().__init__(Q_in, QF_in, R_in, xg_in, QF_start)
        self.plant = plant
        self.n = plant.get_num_pos()
        m = plant.model
        if self.n != 2 or m.H0 is None or not m.is_serial_chain():
            raise ValueError("UrdfCost is defined for 2-link serial arms only (RBDReference.py:262-265; SURVEY F5)")
        if overloading:
            raise NotImplementedError("overloading (op-history tracing) is instrumentation, not offered")
        self.hess_mode = 0

    def _kin(self, q):
        m = self.plant.model
        H = [m.H(j, q[j]) for j in range(2)]
        dH = [m.dH(j, q[j]) for j in range(2)]
        pos = (H[0] @ H[1] @ self.OFFSET)[:2]
        J = np.column_stack(((dH[0] @ H[1] @ self.OFFSET)[:2], (H[0] @ dH[1] @ self.OFFSET)[:2]))
        return pos, J

    def compute_J(self, q):
        """The end-effector Jacobian d p / d q (TrajoptCost.py:398-400 -> RBDReference.Jacobian)."""
        return self._kin(np.asarray(q, dtype=np.float64))[1]

    def dJtotdq(self, q, qd):
        """TrajoptCost.py:460-480: d jacobian_tot_state / d q as a (2n, 2n, 2n) array, from the
        reference's hard-coded 2-link patterns of dJdq / d2Jdq2 (RBDReference.py:219-316)."""
        J = self.compute_J(q)
        n = self.n
        dJdq = np.array([-J[1, :], [-J[1, 1], -J[1, 1]], -J[0, :], [J[0, 1], J[0, 1]]])
        ddJdq = np.array([-J[0, :], [-J[0, 1], -J[0, 1]], -J[1, :], [-J[1, 1], -J[1, 1]]])
        A = np.hstack((dJdq, np.zeros((2 * n, n)))).reshape(n, n, 2 * n)
        Bm = np.hstack((dJdq, ddJdq)).reshape(n, n, 2 * n)
        out = np.zeros((2 * n, 2 * n, 2 * n))
        out[0:n, 0:n, :] = A
        out[n:2 * n, 0:n, :] = Bm
        out[n:2 * n, n:2 * n, :] = A
        return out

    def jacobian_tot_state(self, q, qd):
        """RBDReference.py:313-331 with the hand-coded dJdq pattern (:252-259)."""
        J = self.compute_J(q)
        dJdq = np.array([[-J[1, 0], -J[1, 1]], [-J[1, 1], -J[1, 1]], [-J[0, 0], -J[0, 1]], [J[0, 1], J[0, 1]]])
        J2 = (dJdq @ qd).reshape(2, 2)
        return np.vstack((np.hstack((J, np.zeros((2, 2)))), np.hstack((J2, J))))

    def delta_x(self, x):
        x = np.asarray(x, dtype=np.float64)
        pos, J = self._kin(x[:2])
        return np.concatenate((pos, J @ x[2:])) - self.xg

    def value(self, x, u=None, timestep=None, iter_1=0, iter_2=0, iter_3=0):
        dx = self.delta_x(x)
        cost = 0.5 * (dx @ (self.get_currQ(u, timestep) @ dx))
        if u is not None:
            u = np.asarray(u)
            cost += 0.5 * (u @ (self.R @ u))
        return cost

    def gradient(self, x, u=None, timestep=None, iter_1=0, iter_2=0, iter_3=0):
        x = np.asarray(x, dtype=np.float64)
        top = (self.delta_x(x) @ self.get_currQ(u, timestep)) @ self.jacobian_tot_state(x[:2], x[2:])
        return top if u is None else np.hstack((top, np.asarray(u) @ self.R))

    def hessian(self, x, u=None, timestep=None, iter_1=0, iter_2=0, iter_3=0):
        x = np.asarray(x, dtype=np.float64)
        Jt = self.jacobian_tot_state(x[:2], x[2:])
        hx = (self.get_currQ(u, timestep) @ Jt).T @ Jt
        if u is None:
            return hx
        return np.vstack((np.hstack((hx, np.zeros((4, 2)))), np.hstack((np.zeros((2, 4)), self.R))))
