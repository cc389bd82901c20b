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
