"""Two user plugins for the plugin-hook path, as plain NumPy math shared by the fixture generator (which wraps
them in the REFERENCE's TrajoptCost / TrajoptPlant base classes, tests/golden/make_golden.py run_plugins) and
the tests (which wrap them in this package's classes, tests/test_gpu_plugins.py):

  CoupledCost  a time-varying quadratic cost with an x-u cross term -- G_k is not block-diagonal, so no
               built-in device cost can express it:
                 l_k = 0.5 dx^T Q_k dx + 0.5 u^T R u + u^T M dx,  Q_k = (1 + w k) Q,  terminal 0.5 dx^T QF dx;
  SpringPlant  a 2-joint nonlinear spring-damper system with coupled joints (no URDF):
                 qdd = u - K q - D qd - a sin(q) + s (roll(q) - q)   (elementwise, roll = the other joint).
Both follow the reference's hook signatures (TrajoptCost.py:12-20, TrajoptPlant.py:40-56)."""
import numpy as np

NQ = 2
K_SPRING = np.array([1.5, 0.8])
D_DAMP = np.array([0.3, 0.2])
A_SIN = 2.0
S_COUPLE = 0.4


def spring_qdd(x, u):
    q, qd = x[:NQ], x[NQ:]
    return u - K_SPRING * q - D_DAMP * qd - A_SIN * np.sin(q) + S_COUPLE * (np.roll(q, 1) - q)


def spring_dqdd(x, u):
    """[dqdd/dq | dqdd/dqd | dqdd/du] (NQ x 3 NQ)"""
    q = x[:NQ]
    dq = np.diag(-K_SPRING - A_SIN * np.cos(q) - S_COUPLE) + S_COUPLE * np.roll(np.eye(NQ), 1, axis=1).T
    return np.hstack((dq, np.diag(-D_DAMP), np.eye(NQ)))


def coupled_arrays(nx, nu):
    Q = np.eye(nx)
    QF = 50.0 * np.eye(nx)
    R = 0.2 * np.eye(nu)
    M = 0.05 * np.ones((nu, nx))
    xg = np.zeros(nx)
    xg[0] = 0.5
    return Q, QF, R, M, xg, 0.05


def coupled_value(x, u, k, arrs):
    Q, QF, R, M, xg, w = arrs
    dx = np.asarray(x, dtype=np.float64) - xg
    if u is None:
        return 0.5 * dx @ (QF @ dx)
    u = np.asarray(u, dtype=np.float64)
    return 0.5 * dx @ (((1.0 + w * k) * Q) @ dx) + 0.5 * u @ (R @ u) + u @ (M @ dx)


def coupled_gradient(x, u, k, arrs):
    Q, QF, R, M, xg, w = arrs
    dx = np.asarray(x, dtype=np.float64) - xg
    if u is None:
        return QF @ dx
    u = np.asarray(u, dtype=np.float64)
    return np.concatenate((((1.0 + w * k) * Q) @ dx + M.T @ u, R @ u + M @ dx))


def coupled_hessian(x, u, k, arrs):
    Q, QF, R, M, xg, w = arrs
    if u is None:
        return QF.copy()
    return np.vstack((np.hstack(((1.0 + w * k) * Q, M.T)), np.hstack((M, R))))


def spring_initial(N, dt, seed):
    """q0 ~ U(-1, 1), qd0 = 0, Euler rollout of u = 0"""
    rng = np.random.default_rng(seed)
    x = np.zeros((2 * NQ, N))
    x[:NQ, 0] = rng.uniform(-1.0, 1.0, NQ)
    u = np.zeros((NQ, N - 1))
    for k in range(N - 1):
        x[:, k + 1] = x[:, k] + dt * np.concatenate((x[NQ:, k], spring_qdd(x[:, k], u[:, k])))
    return x, u
