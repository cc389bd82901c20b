"""ctypes binding of libtmpc.so (include/tmpc.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C trajoptmpcreference_amd/csrc``).  There is no CPU fallback: if the
library or a GPU is missing, every solver entry point raises.
"""
import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TMPC_LIBRARY") or os.path.join(_HERE, "libtmpc.so")

LINSYS = {"S": 1, "PCG-J": 2, "PCG-BJ": 3, "PCG-SS": 4, "PCG-0": 5, "N": 6}
SOLVER_ILQR = 16
PRECOND = {"J": 1, "BJ": 2, "SS": 3, "0": 4}

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_up = C.POINTER(C.c_uint64)


class tmpc_options(C.Structure):
    _fields_ = [
        ("exit_tolerance_linSys", C.c_double),
        ("max_iter_linSys", C.c_int32),
        ("max_iter_SQP_DDP", C.c_int32),
        ("exit_tolerance_SQP_DDP", C.c_double),
        ("alpha_factor_SQP_DDP", C.c_double),
        ("alpha_min_SQP_DDP", C.c_double),
        ("rho_factor_SQP_DDP", C.c_double),
        ("rho_min_SQP_DDP", C.c_double),
        ("rho_max_SQP_DDP", C.c_double),
        ("rho_init_SQP_DDP", C.c_double),
        ("expected_reduction_min_SQP_DDP", C.c_double),
        ("expected_reduction_max_SQP_DDP", C.c_double),
        ("merit_mu", C.c_double),
        ("profile", C.c_int32),
        ("max_iter_softConstraints", C.c_int32),
        ("exit_tolerance_softConstraints", C.c_double),
        ("pcg_warm_start", C.c_int32),
        ("precision", C.c_int32),
    ]


LIMIT_MODES = {"QUADRATIC_PENALTY": 1, "AUGMENTED_LAGRANGIAN": 2, "ACTIVE_SET": 3, "FULL_SET": 4}


class tmpc_box_limits(C.Structure):
    _fields_ = [
        ("mode", C.c_int32 * 3), ("reserved", C.c_int32),
        ("lb", (C.c_double * 8) * 3), ("ub", (C.c_double * 8) * 3),
        ("mu_init", C.c_double * 3), ("mu_factor", C.c_double * 3), ("mu_max", C.c_double * 3),
        ("phi_init", C.c_double * 3), ("phi_factor", C.c_double * 3),
    ]


class tmpc_trace(C.Structure):
    _fields_ = [
        ("iteration", _ip), ("line_search_iteration", _ip), ("alpha", _dp), ("rho", _dp), ("J", _dp),
        ("c", _dp), ("merit", _dp), ("D", _dp), ("reduction_ratio", _dp), ("succeeded_line_search", _ip),
        ("pcg_iters", _ip), ("singular", _ip), ("hard_active", _up),
    ]


class tmpc_stream(C.Structure):
    """continuous batching (tmpc_*_solve_stream_device): device arrays, include/tmpc.h"""
    _fields_ = [("problems", C.c_int32), ("slots", C.c_int32), ("period", C.c_int32), ("substreams", C.c_int32),
                ("x_in", C.c_void_p), ("u_in", C.c_void_p), ("x_out", C.c_void_p), ("u_out", C.c_void_p),
                ("status", C.c_void_p), ("trace", tmpc_trace)]


TRACE_FIELDS = [("iteration", np.int32), ("line_search_iteration", np.int32), ("alpha", np.float64),
                ("rho", np.float64), ("J", np.float64), ("c", np.float64), ("merit", np.float64),
                ("D", np.float64), ("reduction_ratio", np.float64), ("succeeded_line_search", np.int32),
                ("pcg_iters", np.int32), ("singular", np.int32)]


# every symbol include/tmpc.h declares, with its ctypes signature
SIGNATURES = {
    "tmpc_abi_version": (C.c_int, []),
    "tmpc_device_count": (C.c_int, [_ip]),
    "tmpc_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "tmpc_destroy": (None, [C.c_void_p]),
    "tmpc_last_error": (C.c_char_p, [C.c_void_p]),
    "tmpc_set_model": (C.c_int, [C.c_void_p, C.c_int, _ip, _ip, _ip, _dp, _dp, _dp, _dp, C.c_double]),
    "tmpc_set_cost_quadratic": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dp, _dp, _dp, _dp, C.c_int32]),
    "tmpc_set_cost_ee": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dp, _dp, _dp, _dp, C.c_int32, _dp, _dp, _dp]),
    "tmpc_default_options": (None, [C.POINTER(tmpc_options)]),
    "tmpc_set_options": (C.c_int, [C.c_void_p, C.POINTER(tmpc_options)]),
    "tmpc_set_box_limits": (C.c_int, [C.c_void_p, C.POINTER(tmpc_box_limits)]),
    "tmpc_set_soft_state": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dp, _dp, _dp]),
    "tmpc_get_soft_state": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dp, _dp, _dp]),
    "tmpc_sqp_solve_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_int, _dp, _dp, _ip, _ip, _ip,
                                       _ip, C.POINTER(tmpc_trace)]),
    "tmpc_sqp_solve_batch_device": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_int, C.c_void_p,
                                              C.c_void_p, _ip, _ip]),
    "tmpc_ilqr_solve_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, _dp, _dp, _ip, _ip, _ip, _ip,
                                        C.POINTER(tmpc_trace)]),
    "tmpc_ilqr_solve_batch_device": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_void_p,
                                               _ip, _ip]),
    "tmpc_sqp_solve_stream_device": (C.c_int, [C.c_void_p, C.c_int, C.c_double, C.c_int, C.POINTER(tmpc_stream)]),
    "tmpc_ilqr_solve_stream_device": (C.c_int, [C.c_void_p, C.c_int, C.c_double, C.POINTER(tmpc_stream)]),
    "tmpc_mpc_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int, _dp, _dp, _dp, _dp,
                                 _ip, _ip]),
    "tmpc_mpc_batch_device": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "tmpc_rollout_batch_device": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_void_p]),
    "tmpc_fd_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_double, _dp, _dp, _dp, _dp, _dp]),
    "tmpc_fd_grad_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_double, _dp, _dp, _dp, _dp, _dp]),
    "tmpc_qp_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_int, _dp, _dp, _dp, _dp, _dp, _dp, _ip,
                                _dp, _dp, _dp, _dp]),
    "tmpc_qp_blocks_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp,
                                       _dp, _dp, _dp, _dp, _ip, _dp, _dp, _dp]),
    "tmpc_qp_blocks_banded_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp,
                                              _dp, _dp, _ip, _ip, _dp, _dp, C.c_int, _dp, _dp, _ip, _dp, _ip]),
    "tmpc_qp_hard_info": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _ip, _ip, _up, _dp, _dp, _dp, _ip]),
    "tmpc_hard_pcg_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, _ip, C.c_int, _dp, _dp,
                                      C.c_double, C.c_int, _dp, _ip]),
    "tmpc_pcg_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp, _dp, C.c_double,
                                 C.c_int, _dp, _ip, _dp, _dp, _dp]),
    "tmpc_pcg_dense_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _dp, _dp, _dp, C.c_int, C.c_int, _dp,
                                       C.c_double, C.c_int, _dp, _ip, _dp, _dp, _dp]),
    "tmpc_device_alloc": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    "tmpc_device_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "tmpc_memcpy_h2d": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "tmpc_memcpy_d2h": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "tmpc_memcpy_d2d": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "tmpc_synchronize": (C.c_int, [C.c_void_p]),
    "tmpc_kernel_stats": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_double)]),
    "tmpc_reset_stats": (C.c_int, [C.c_void_p]),
    "tmpc_solve_counters": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "tmpc_kernel_bytes": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_double)]),
    "tmpc_comm_get_unique_id": (C.c_int, [C.c_void_p]),
    "tmpc_comm_create": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]),
    "tmpc_comm_destroy": (None, [C.c_void_p]),
    "tmpc_comm_size": (C.c_int, [C.c_void_p, _ip, _ip]),
    "tmpc_comm_broadcast": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]),
    "tmpc_comm_allgather": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "tmpc_comm_allreduce_max_f64": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "tmpc_comm_barrier": (C.c_int, [C.c_void_p]),
}
COMM_ID_BYTES = 128

_lib = None
_lib_lock = threading.Lock()


class NativeError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH):
    """Load libtmpc.so and bind every exported symbol (raises if missing)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NativeError(f"{path} not found: build it with __graft_entry__.build() "
                              "(or `make -C trajoptmpcreference_amd/csrc`); there is no CPU fallback")
        lib = C.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def device_count() -> int:
    lib = load_library()
    n = C.c_int32(0)
    lib.tmpc_device_count(C.byref(n))
    return int(n.value)


def _ptr(a):
    if a is None:
        return None
    if a.dtype == np.float64:
        return a.ctypes.data_as(_dp)
    if a.dtype == np.int32:
        return a.ctypes.data_as(_ip)
    if a.dtype == np.uint64:
        return a.ctypes.data_as(_up)
    raise TypeError(a.dtype)


def _c64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class Context:
    """One libtmpc context (one GPU, one HIP stream)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.tmpc_create(int(device), C.byref(h))
        if rc != 0:
            n = device_count()
            raise NativeError(f"tmpc_create(device={device}) failed (code {rc}; {n} HIP device(s) visible). "
                              "The solver runs on an AMD GPU only.")
        self.h = h
        self.device = device
        self.model = None
        self.nx = self.nu = None
        self.options = tmpc_options()
        self.lib.tmpc_default_options(C.byref(self.options))

    def close(self):
        if getattr(self, "h", None):
            self.lib.tmpc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check_traj(self, x, u, N):
        """x [B][nx][N], u [B][nu][N-1] with nx / nu of the loaded model: the library copies
        B*nx*N and B*nu*(N-1) doubles in and out of these buffers."""
        if self.model is None:
            raise NativeError("no model: call set_model first")
        n = self.model.n
        if x.ndim != 3 or u.ndim != 3 or x.shape[0] != u.shape[0] or x.shape[1:] != (2 * n, N) \
                or u.shape[1:] != (n, N - 1):
            raise ValueError(f"expected x [B][{2 * n}][{N}] and u [B][{n}][{N - 1}] for a {n}-joint model, "
                             f"got {x.shape} and {u.shape}")

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.tmpc_last_error(self.h)
            raise NativeError(f"{what}: {msg.decode() if msg else 'error'} (code {rc})")

    # ---------------------------------------------------------------- configuration
    def set_model(self, model, gravity=-9.81):
        n = model.n
        saxis = np.array([int(np.argmax(model.S[j])) for j in range(n)], dtype=np.int32)
        self._check(self.lib.tmpc_set_model(
            self.h, n, _ptr(np.ascontiguousarray(model.parent, dtype=np.int32)),
            _ptr(np.ascontiguousarray(model.jtype, dtype=np.int32)), _ptr(saxis),
            _ptr(_c64(model.X0)), _ptr(_c64(model.Xa)), _ptr(_c64(model.Xb)), _ptr(_c64(model.I)), float(gravity)),
            "tmpc_set_model")
        self.model = model

    def set_cost_quadratic(self, Q, QF, R, xg, QF_start=None):
        Q, QF, R, xg = _c64(Q), _c64(QF), _c64(R), _c64(xg).reshape(-1)
        self.nx, self.nu = Q.shape[0], R.shape[0]
        self._check(self.lib.tmpc_set_cost_quadratic(self.h, self.nx, self.nu, _ptr(Q), _ptr(QF), _ptr(R), _ptr(xg),
                                                     -1 if QF_start is None else int(QF_start)),
                    "tmpc_set_cost_quadratic")

    def set_cost_ee(self, Q, QF, R, xg, QF_start, H0, Ha, Hb):
        """UrdfCost (TrajoptCost.py:371-569): H0/Ha/Hb are the 2 joints' homogeneous
        transform coefficients (RobotModel.H0/Ha/Hb[:2])."""
        Q, QF, R, xg = _c64(Q), _c64(QF), _c64(R), _c64(xg).reshape(-1)
        H0, Ha, Hb = _c64(H0), _c64(Ha), _c64(Hb)
        self.nx, self.nu = Q.shape[0], R.shape[0]
        self._check(self.lib.tmpc_set_cost_ee(self.h, self.nx, self.nu, _ptr(Q), _ptr(QF), _ptr(R), _ptr(xg),
                                              -1 if QF_start is None else int(QF_start), _ptr(H0), _ptr(Ha),
                                              _ptr(Hb)), "tmpc_set_cost_ee")

    def set_options(self, **kw):
        for k, v in kw.items():
            if not hasattr(self.options, k):
                raise KeyError(k)
            setattr(self.options, k, v)
        self._check(self.lib.tmpc_set_options(self.h, C.byref(self.options)), "tmpc_set_options")

    def set_box_limits(self, limits):
        """limits: None, or {type: dict(mode=..., lb=[n], ub=[n], options=...)} with type in
        joint / velocity / torque (TrajoptConstraint.set_*_limits)."""
        if not limits:
            self._check(self.lib.tmpc_set_box_limits(self.h, None), "tmpc_set_box_limits")
            return
        L = tmpc_box_limits()
        n = self.model.n
        for t, name in enumerate(("joint", "velocity", "torque")):
            spec = limits.get(name)
            if spec is None:
                continue
            L.mode[t] = LIMIT_MODES[spec["mode"]]
            lb = np.broadcast_to(np.asarray(spec["lb"], dtype=np.float64), (n,))
            ub = np.broadcast_to(np.asarray(spec["ub"], dtype=np.float64), (n,))
            # the ABI rows hold 8 joints; limits on a wider model are refused by the solve (check_ready)
            for i in range(min(n, len(L.lb[t]))):
                L.lb[t][i] = float(lb[i])
                L.ub[t][i] = float(ub[i])
            o = spec.get("options", {})
            L.mu_init[t] = o.get("quadratic_penalty_mu_init", 1e-2)
            L.mu_factor[t] = o.get("quadratic_penalty_mu_factor", 10.0)
            L.mu_max[t] = o.get("quadratic_penalty_mu_max", 1e12)
            L.phi_init[t] = o.get("augmentated_lagrangian_phi_init", 1e-2)
            L.phi_factor[t] = o.get("augmentated_lagrangian_phi_factor", 10.0)
        self._check(self.lib.tmpc_set_box_limits(self.h, C.byref(L)), "tmpc_set_box_limits")

    def set_soft_state(self, B, N, mu=None, lam=None, phi=None):
        """[B][N][6n] arrays (None: defaults)."""
        arrs = [None if a is None else _c64(a) for a in (mu, lam, phi)]
        shape = (int(B), int(N), 6 * self.model.n)
        for a in arrs:
            if a is not None and a.shape != shape:
                raise ValueError(f"soft-constraint state must be {shape}, got {a.shape}")
        self._check(self.lib.tmpc_set_soft_state(self.h, int(B), int(N), *[_ptr(a) for a in arrs]),
                    "tmpc_set_soft_state")

    def get_soft_state(self, B, N):
        shape = (B, N, 6 * self.model.n)
        mu, lam, phi = np.zeros(shape), np.zeros(shape), np.zeros(shape)
        self._check(self.lib.tmpc_get_soft_state(self.h, int(B), int(N), _ptr(mu), _ptr(lam), _ptr(phi)),
                    "tmpc_get_soft_state")
        return mu, lam, phi

    # ---------------------------------------------------------------- solves
    def _trace_arrays(self, B, N=None, hard_active=False):
        W = int(self.options.max_iter_SQP_DDP) + 1
        arrays = {}
        for name, dt_ in TRACE_FIELDS:
            arrays[name] = np.zeros((B, W), dtype=dt_)
        if hard_active:
            arrays["hard_active"] = np.zeros((B, W, N), dtype=np.uint64)
        return arrays, tmpc_trace(**{k: _ptr(v) for k, v in arrays.items()})

    def sqp_solve_batch(self, x, u, N, dt, method="PCG-SS", with_trace=True, hard_active=False):
        """x [B][nx][N], u [B][nu][N-1] -> dict of results (arrays per problem).  hard_active: also the
        per-QP active-set bitmasks of the hard box limits, trace["hard_active"] [B][max_iter+1][N]."""
        x = _c64(x).copy()
        u = _c64(u).copy()
        self._check_traj(x, u, N)
        B = x.shape[0]
        out = {k: np.zeros(B, dtype=np.int32) for k in ("exit_sqp", "exit_soft", "outer_iter", "sqp_iter")}
        arrays, tr = self._trace_arrays(B, N, hard_active) if with_trace else ({}, None)
        self._check(self.lib.tmpc_sqp_solve_batch(
            self.h, B, int(N), float(dt), LINSYS[method], _ptr(x), _ptr(u), _ptr(out["exit_sqp"]),
            _ptr(out["exit_soft"]), _ptr(out["outer_iter"]), _ptr(out["sqp_iter"]),
            C.byref(tr) if tr is not None else None), "tmpc_sqp_solve_batch")
        out.update(x=x, u=u, trace=arrays)
        return out

    def ilqr_solve_batch(self, x, u, N, dt, with_trace=True):
        """Batched iLQR (oracle/ilqr.py): x [B][nx][N] (only x[:, :, 0] is read), u [B][nu][N-1]."""
        x = _c64(x).copy()
        u = _c64(u).copy()
        self._check_traj(x, u, N)
        B = x.shape[0]
        out = {k: np.zeros(B, dtype=np.int32) for k in ("exit_code", "exit_soft", "outer_iter", "iter")}
        arrays, tr = self._trace_arrays(B) if with_trace else ({}, None)
        self._check(self.lib.tmpc_ilqr_solve_batch(
            self.h, B, int(N), float(dt), _ptr(x), _ptr(u), _ptr(out["exit_code"]), _ptr(out["exit_soft"]),
            _ptr(out["outer_iter"]), _ptr(out["iter"]), C.byref(tr) if tr is not None else None),
            "tmpc_ilqr_solve_batch")
        out.update(x=x, u=u, trace=arrays)
        return out

    def mpc_batch(self, x, u, N, dt, solver, steps):
        """Receding-horizon loop (oracle/mpc.py); solver = "iLQR" or an SQP method name."""
        x = _c64(x).copy()
        u = _c64(u).copy()
        self._check_traj(x, u, N)
        B, nx, _ = x.shape
        nu = u.shape[1]
        xe = np.zeros((B, nx, steps + 1))
        ue = np.zeros((B, nu, steps))
        codes = np.zeros((B, steps), dtype=np.int32)
        iters = np.zeros((B, steps), dtype=np.int32)
        sid = SOLVER_ILQR if solver == "iLQR" else LINSYS[solver]
        self._check(self.lib.tmpc_mpc_batch(self.h, B, int(N), float(dt), sid, int(steps), _ptr(x), _ptr(u), _ptr(xe),
                                            _ptr(ue), _ptr(codes), _ptr(iters)), "tmpc_mpc_batch")
        return dict(x=x, u=u, x_exec=xe, u_exec=ue, exit_codes=codes, iters=iters)

    def mpc_batch_device(self, B, N, dt, solver, steps, d_x, d_u, d_xe, d_ue, d_codes, d_iters):
        sid = SOLVER_ILQR if solver == "iLQR" else LINSYS[solver]
        self._check(self.lib.tmpc_mpc_batch_device(self.h, B, int(N), float(dt), sid, int(steps), d_x, d_u, d_xe, d_ue,
                                                   d_codes, d_iters), "tmpc_mpc_batch_device")

    def ilqr_solve_batch_device(self, B, N, dt, d_x, d_u, want_status=False):
        ex = np.zeros(B, dtype=np.int32) if want_status else None
        it = np.zeros(B, dtype=np.int32) if want_status else None
        self._check(self.lib.tmpc_ilqr_solve_batch_device(self.h, B, int(N), float(dt), d_x, d_u, _ptr(ex), _ptr(it)),
                    "tmpc_ilqr_solve_batch_device")
        return ex, it

    def fd_batch(self, x, u, dt=0.0, want_minv=True):
        x, u = _c64(x), _c64(u)
        K, nx = x.shape
        n = nx // 2
        xn = np.zeros((K, nx))
        qdd = np.zeros((K, n))
        Mi = np.zeros((K, n, n)) if want_minv else None
        self._check(self.lib.tmpc_fd_batch(self.h, K, float(dt), _ptr(x), _ptr(u), _ptr(xn), _ptr(qdd), _ptr(Mi)),
                    "tmpc_fd_batch")
        return xn, qdd, Mi

    def fd_grad_batch(self, x, u, dt):
        x, u = _c64(x), _c64(u)
        K, nx = x.shape
        n = nx // 2
        A = np.zeros((K, nx, nx))
        Bm = np.zeros((K, nx, n))
        dq = np.zeros((K, n, 3 * n))
        self._check(self.lib.tmpc_fd_grad_batch(self.h, K, float(dt), _ptr(x), _ptr(u), _ptr(A), _ptr(Bm), _ptr(dq)),
                    "tmpc_fd_grad_batch")
        return A, Bm, dq

    def qp_batch(self, x, u, N, dt, rho, method="PCG-SS", want_blocks=True, guess=None, xs=None):
        """guess [B][N nx]: the PCG initial iterate (solveKKTSystem_Schur's options['guess']); xs [B][nx]: the
        SQP's initial state (default x[:, :, 0]).
        With hard box limits set, want_blocks must be False and the lambda part of dxul holds the
        dynamics-row multipliers only (include/tmpc.h)."""
        x, u = _c64(x), _c64(u)
        self._check_traj(x, u, N)
        B, nx, _ = x.shape
        nu = u.shape[1]
        if guess is not None:
            guess = _c64(guess).reshape(B, N * nx)
        if xs is not None:
            xs = _c64(np.broadcast_to(np.asarray(xs, dtype=np.float64), (B, nx)))
        rho = _c64(np.broadcast_to(np.asarray(rho, dtype=np.float64), (B,)))
        L = (nx + nu) * (N - 1) + nx + nx * N
        dxul = np.zeros((B, L))
        iters = np.zeros(B, dtype=np.int32)
        Sd = np.zeros((B, N, nx, nx)) if want_blocks else None
        Sl = np.zeros((B, N - 1, nx, nx)) if want_blocks else None
        g = np.zeros((B, N * nx)) if want_blocks else None
        Pd = np.zeros((B, N, nx, nx)) if want_blocks else None
        self._check(self.lib.tmpc_qp_batch(self.h, B, int(N), float(dt), LINSYS[method], _ptr(rho), _ptr(x), _ptr(u),
                                           _ptr(xs), _ptr(guess), _ptr(dxul), _ptr(iters), _ptr(Sd), _ptr(Sl), _ptr(g),
                                           _ptr(Pd)),
                    "tmpc_qp_batch")
        return dict(dxul=dxul, pcg_iters=iters, S_diag=Sd, S_lo=Sl, gamma=g, P_diag=Pd)

    def qp_blocks_batch(self, G, g, A, Bm, c, rho, method="PCG-SS", guess=None, want_blocks=False):
        """solveKKTSystem(_Schur) on caller-formed blocks (tmpc_qp_blocks_batch, the plugin-hook QP):
        G [B][N][n][n] (without rho; knot N-1 in the top-left nx x nx corner), g [B][N][n], A [B][N-1][nx][nx],
        Bm [B][N-1][nx][nu], c [B][N][nx], rho [B] -> dict(dxul [B][n(N-1)+nx+nx N], pcg_iters [B], and with
        want_blocks S_diag / S_lo / gamma)."""
        G, g, A, Bm, c = _c64(G), _c64(g), _c64(A), _c64(Bm), _c64(c)
        B, N, n, _ = G.shape
        nx, nu = A.shape[2], Bm.shape[3]
        if g.shape != (B, N, n) or A.shape != (B, N - 1, nx, nx) or Bm.shape != (B, N - 1, nx, nu) \
                or c.shape != (B, N, nx) or n != nx + nu:
            raise ValueError(f"inconsistent block shapes G {G.shape} g {g.shape} A {A.shape} B {Bm.shape} c {c.shape}")
        rho = _c64(np.broadcast_to(np.asarray(rho, dtype=np.float64), (B,)))
        if guess is not None:
            guess = _c64(guess).reshape(B, N * nx)
        dxul = np.zeros((B, n * (N - 1) + nx + nx * N))
        iters = np.zeros(B, dtype=np.int32)
        Sd = np.zeros((B, N, nx, nx)) if want_blocks else None
        Sl = np.zeros((B, N - 1, nx, nx)) if want_blocks else None
        gam = np.zeros((B, N * nx)) if want_blocks else None
        self._check(self.lib.tmpc_qp_blocks_batch(self.h, B, N, nx, nu, LINSYS[method], _ptr(G), _ptr(g), _ptr(A),
                                                  _ptr(Bm), _ptr(c), _ptr(rho), _ptr(guess), _ptr(dxul), _ptr(iters),
                                                  _ptr(Sd), _ptr(Sl), _ptr(gam)), "tmpc_qp_blocks_batch")
        return dict(dxul=dxul, pcg_iters=iters, S_diag=Sd, S_lo=Sl, gamma=gam)

    def qp_blocks_banded_batch(self, G, g, A, Bm, c, rho, rows, method="PCG-SS"):
        """tmpc_qp_blocks_banded_batch: the plugin-hook QP with hard box rows and / or past 1024 rows.  G, g, A, Bm,
        c, rho as qp_blocks_batch; rows[b][k] = [(column in [x_k; u_k], sign, value), ...] of knot k of problem b
        in the reference's row order (sign +1 / -1, 0 for an inactive FULL_SET row).  Returns dict(dxul,
        pcg_iters, lambda_hard [B][N][rmax], singular)."""
        G, g, A, Bm, c = _c64(G), _c64(g), _c64(A), _c64(Bm), _c64(c)
        B, N, n, _ = G.shape
        nx, nu = A.shape[2], Bm.shape[3]
        rmax = max([len(rk) for rb in rows for rk in rb] + [0])
        rb_ = max(rmax, 1)
        cnt = np.zeros((B, N), dtype=np.int32)
        col = np.zeros((B, N, rb_), dtype=np.int32)
        sgn = np.zeros((B, N, rb_))
        val = np.zeros((B, N, rb_))
        for b in range(B):
            for k in range(N):
                cnt[b, k] = len(rows[b][k])
                for r, (cl, sg, v) in enumerate(rows[b][k]):
                    col[b, k, r], sgn[b, k, r], val[b, k, r] = cl, sg, v
        rho = _c64(np.broadcast_to(np.asarray(rho, dtype=np.float64), (B,)))
        dxul = np.zeros((B, n * (N - 1) + nx + nx * N))
        iters = np.zeros(B, dtype=np.int32)
        lam_h = np.zeros((B, N, rb_))
        sing = np.zeros(B, dtype=np.int32)
        if rmax > 0:
            col, sgn, val = np.ascontiguousarray(col[:, :, :rmax]), np.ascontiguousarray(sgn[:, :, :rmax]), \
                np.ascontiguousarray(val[:, :, :rmax])
        self._check(self.lib.tmpc_qp_blocks_banded_batch(
            self.h, B, N, nx, nu, LINSYS[method], _ptr(G), _ptr(g), _ptr(A), _ptr(Bm), _ptr(c), _ptr(cnt), _ptr(col),
            _ptr(sgn), _ptr(val), int(rmax), _ptr(rho), _ptr(dxul), _ptr(iters), _ptr(lam_h), _ptr(sing)),
            "tmpc_qp_blocks_banded_batch")
        return dict(dxul=dxul, pcg_iters=iters, lambda_hard=lam_h, singular=sing)

    def qp_hard_info(self, B, N):
        """Hard-limit detail of the last qp_batch (tmpc_qp_hard_info): dict with dim [B], active [B][N]
        (uint64 bitmasks), lambda_hard [B][N][6n], S_band [B][dmax][2W+1], gamma [B][dmax], singular [B], W."""
        sizes = np.zeros(2, dtype=np.int32)
        self._check(self.lib.tmpc_qp_hard_info(self.h, int(B), int(N), _ptr(sizes), None, None, None, None, None,
                                               None), "tmpc_qp_hard_info")
        dmax, W = int(sizes[0]), int(sizes[1])
        out = dict(dim=np.zeros(B, dtype=np.int32), active=np.zeros((B, N), dtype=np.uint64),
                   lambda_hard=np.zeros((B, N, 6 * (self.model.n if self.model is not None else 0))), S_band=np.zeros((B, dmax, 2 * W + 1)),
                   gamma=np.zeros((B, dmax)), singular=np.zeros(B, dtype=np.int32))
        self._check(self.lib.tmpc_qp_hard_info(self.h, int(B), int(N), _ptr(sizes), _ptr(out["dim"]),
                                               _ptr(out["active"]), _ptr(out["lambda_hard"]), _ptr(out["S_band"]),
                                               _ptr(out["gamma"]), _ptr(out["singular"])), "tmpc_qp_hard_info")
        out["W"] = W
        return out

    def hard_pcg_batch(self, S_band, gamma, dim, nx, precond="SS", tol=1e-6, max_iter=100):
        """The hard-limit QP's banded PCG (tmpc_hard_pcg_batch) on given S_band [B][dmax][2W+1]."""
        S_band, gamma = _c64(S_band), _c64(gamma)
        B, dmax, BW = S_band.shape
        dim = np.ascontiguousarray(dim, dtype=np.int32)
        lam = np.zeros((B, dmax))
        it = np.zeros(B, dtype=np.int32)
        self._check(self.lib.tmpc_hard_pcg_batch(self.h, B, int(nx), dmax, (BW - 1) // 2, _ptr(dim), PRECOND[precond],
                                                 _ptr(S_band), _ptr(gamma), float(tol), int(max_iter), _ptr(lam),
                                                 _ptr(it)), "tmpc_hard_pcg_batch")
        return lam, it

    def pcg_batch(self, S_diag, S_lo, gamma, precond="SS", S_up=None, guess=None, tol=1e-6, max_iter=100,
                  trace=True):
        S_diag, gamma = _c64(S_diag), _c64(gamma)
        B, N, nx, _ = S_diag.shape
        S_lo = _c64(S_lo) if N > 1 else np.zeros((B, 1, nx, nx))
        S_up = _c64(S_up) if S_up is not None else None
        guess = _c64(guess) if guess is not None else None
        lam = np.zeros((B, N * nx))
        it = np.zeros(B, dtype=np.int32)
        tn = np.full((B, max_iter + 1), np.nan) if trace else None
        tr = np.full((B, max_iter + 1), np.nan) if trace else None
        Pd = np.zeros((B, N, nx, nx))
        self._check(self.lib.tmpc_pcg_batch(self.h, B, N, nx, PRECOND[precond], _ptr(S_diag), _ptr(S_lo), _ptr(S_up),
                                            _ptr(gamma), _ptr(guess), float(tol), int(max_iter), _ptr(lam), _ptr(it),
                                            _ptr(tn), _ptr(tr), _ptr(Pd)), "tmpc_pcg_batch")
        return lam, it, tn, tr, Pd

    def pcg_dense_batch(self, A, b, Pinv=None, precond="SS", nx=1, guess=None, tol=1e-6, max_iter=100, trace=True,
                        want_pinv=False):
        """tmpc_pcg_dense_batch: PCG.pcg on dense systems A [B][D][D], b [B][D] with the preconditioner matrix
        Pinv [B][D][D] (None: PCG.solve's block preconditioner `precond` of block size nx, built on the
        device).  Returns x [B][D], iters [B], trace_nu, trace_res ([B][max_iter+1] or None) and the
        preconditioner matrix used (want_pinv, else None)."""
        A, b = _c64(A), _c64(b)
        B, D = b.shape
        if A.shape != (B, D, D):
            raise ValueError(f"A must be [B][D][D] = {(B, D, D)}, got {A.shape}")
        Pinv = _c64(Pinv) if Pinv is not None else None
        if Pinv is not None and Pinv.shape != (B, D, D):
            raise ValueError(f"Pinv must be [B][D][D] = {(B, D, D)}, got {Pinv.shape}")
        guess = _c64(guess) if guess is not None else None
        x = np.zeros((B, D))
        it = np.zeros(B, dtype=np.int32)
        tn = np.full((B, max_iter + 1), np.nan) if trace else None
        tr = np.full((B, max_iter + 1), np.nan) if trace else None
        Po = np.zeros((B, D, D)) if want_pinv else None
        self._check(self.lib.tmpc_pcg_dense_batch(self.h, B, D, _ptr(A), _ptr(b), _ptr(Pinv), PRECOND[precond],
                                                  int(nx), _ptr(guess), float(tol), int(max_iter), _ptr(x), _ptr(it),
                                                  _ptr(tn), _ptr(tr), _ptr(Po)), "tmpc_pcg_dense_batch")
        return x, it, tn, tr, Po

    # ---------------------------------------------------------------- device memory (bench)
    def alloc(self, nbytes):
        p = C.c_void_p()
        self._check(self.lib.tmpc_device_alloc(self.h, int(nbytes), C.byref(p)), "tmpc_device_alloc")
        return p

    def free(self, p):
        self._check(self.lib.tmpc_device_free(self.h, p), "tmpc_device_free")

    def h2d(self, dst, arr):
        arr = np.ascontiguousarray(arr)
        self._check(self.lib.tmpc_memcpy_h2d(self.h, dst, arr.ctypes.data_as(C.c_void_p), arr.nbytes), "h2d")

    def d2h(self, arr, src, offset=0):
        """device -> host copy of arr.nbytes bytes starting `offset` bytes into the device buffer src"""
        if offset:
            src = C.c_void_p((src.value if isinstance(src, C.c_void_p) else int(src)) + int(offset))
        self._check(self.lib.tmpc_memcpy_d2h(self.h, arr.ctypes.data_as(C.c_void_p), src, arr.nbytes), "d2h")

    def d2d(self, dst, src, nbytes):
        self._check(self.lib.tmpc_memcpy_d2d(self.h, dst, src, int(nbytes)), "d2d")

    def synchronize(self):
        self._check(self.lib.tmpc_synchronize(self.h), "tmpc_synchronize")

    def rollout_device(self, B, N, dt, d_x, d_u):
        self._check(self.lib.tmpc_rollout_batch_device(self.h, B, N, float(dt), d_x, d_u), "tmpc_rollout_batch_device")

    def sqp_solve_batch_device(self, B, N, dt, d_x, d_u, method="PCG-SS", want_status=False):
        ex = np.zeros(B, dtype=np.int32) if want_status else None
        it = np.zeros(B, dtype=np.int32) if want_status else None
        self._check(self.lib.tmpc_sqp_solve_batch_device(self.h, B, int(N), float(dt), LINSYS[method], d_x, d_u,
                                                         _ptr(ex), _ptr(it)), "tmpc_sqp_solve_batch_device")
        return ex, it

    def solve_stream_device(self, solver, P, slots, N, dt, d_x_in, d_u_in, period, d_x_out=None, d_u_out=None,
                            d_status=None, d_trace=None, substreams=1):
        """Continuous batching (tmpc_sqp_solve_stream_device / tmpc_ilqr_solve_stream_device): P problems
        through `slots` resident slots, problem p from input p % period; device pointers (d_trace: dict of
        trace field -> device pointer [P][max_iter+1]); substreams: K concurrent sub-streams."""
        st = tmpc_stream(problems=int(P), slots=int(slots), period=int(period), substreams=int(substreams), x_in=d_x_in,
                         u_in=d_u_in, x_out=d_x_out, u_out=d_u_out, status=d_status)
        for name, dt_ in TRACE_FIELDS:
            p = (d_trace or {}).get(name)
            if p is not None:
                setattr(st.trace, name, C.cast(p, _ip if dt_ == np.int32 else _dp))
        if solver == "iLQR":
            self._check(self.lib.tmpc_ilqr_solve_stream_device(self.h, int(N), float(dt), C.byref(st)),
                        "tmpc_ilqr_solve_stream_device")
        else:
            self._check(self.lib.tmpc_sqp_solve_stream_device(self.h, int(N), float(dt), LINSYS[solver], C.byref(st)),
                        "tmpc_sqp_solve_stream_device")

    def solve_stream(self, x, u, N, dt, solver="PCG-SS", slots=64, copies=1, with_trace=True, substreams=1):
        """Host convenience of solve_stream_device: problems x [P0][nx][N], u [P0][nu][N-1], each solved
        `copies` times (stream problem p = input p % P0) through `slots` slots.  Returns x, u [P][..],
        status fields (exit, iters, exit_soft, outer_iter) [P] and the trace [P][max_iter+1]."""
        x, u = _c64(x), _c64(u)
        self._check_traj(x, u, N)
        P0 = x.shape[0]
        P = P0 * int(copies)
        W = int(self.options.max_iter_SQP_DDP) + 1
        bufs = []
        try:
            def dev(nbytes):
                p = self.alloc(max(8, nbytes))
                bufs.append(p)
                return p
            dxi, dui = dev(x.nbytes), dev(u.nbytes)
            self.h2d(dxi, x)
            self.h2d(dui, u)
            dxo, duo, dst = dev(x.nbytes * copies), dev(u.nbytes * copies), dev(P * 4 * 4)
            dtr = {name: dev(P * W * np.dtype(dt_).itemsize) for name, dt_ in TRACE_FIELDS} if with_trace else None
            self.solve_stream_device(solver, P, slots, N, dt, dxi, dui, P0, dxo, duo, dst, dtr, substreams)
            xo = np.empty((P,) + x.shape[1:])
            uo = np.empty((P,) + u.shape[1:])
            status = np.empty((P, 4), dtype=np.int32)
            self.d2h(xo, dxo)
            self.d2h(uo, duo)
            self.d2h(status, dst)
            trace = {}
            if with_trace:
                for name, dt_ in TRACE_FIELDS:
                    trace[name] = np.empty((P, W), dtype=dt_)
                    self.d2h(trace[name], dtr[name])
        finally:
            for p in bufs:
                self.free(p)
        return dict(x=xo, u=uo, exit=status[:, 0].copy(), iters=status[:, 1].copy(), exit_soft=status[:, 2].copy(),
                    outer_iter=status[:, 3].copy(), trace=trace)

    def kernel_stats(self, name):
        n = C.c_int64(0)
        ms = C.c_double(0.0)
        self._check(self.lib.tmpc_kernel_stats(self.h, name.encode(), C.byref(n), C.byref(ms)), "tmpc_kernel_stats")
        return int(n.value), float(ms.value)

    def kernel_bytes(self, name):
        """Algorithmic HBM bytes a counting kernel ("hard_pcg") moved since reset_stats (tmpc_kernel_bytes)."""
        v = C.c_double(0.0)
        self._check(self.lib.tmpc_kernel_bytes(self.h, name.encode(), C.byref(v)), "tmpc_kernel_bytes")
        return float(v.value)

    def solve_counters(self):
        """[problem-QPs, PCG iterations, gradient recomputations, line-search trials per QP] of the last solve."""
        c = (C.c_int64 * 4)()
        self._check(self.lib.tmpc_solve_counters(self.h, c), "tmpc_solve_counters")
        return [int(v) for v in c]

    def reset_stats(self):
        self._check(self.lib.tmpc_reset_stats(self.h), "tmpc_reset_stats")


def comm_unique_id() -> bytes:
    """ncclGetUniqueId (rank 0, before the id is shared with the other ranks)."""
    lib = load_library()
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    if lib.tmpc_comm_get_unique_id(buf) != 0:
        raise NativeError("tmpc_comm_get_unique_id failed (RCCL)")
    return bytes(buf)


class Comm:
    """RCCL communicator over the GPUs of a node (tmpc_comm_*, include/tmpc.h): one rank per
    process / GPU.  Host-array helpers stage through device memory of the context."""

    def __init__(self, ctx: Context, nranks: int, rank: int, uid: bytes):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"RCCL unique id must be {COMM_ID_BYTES} bytes")
        self.ctx, self.lib = ctx, ctx.lib
        self.world, self.rank = int(nranks), int(rank)
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        ctx._check(self.lib.tmpc_comm_create(ctx.h, self.world, self.rank, buf, C.byref(h)), "tmpc_comm_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.tmpc_comm_destroy(self.h)
            self.h = None

    def barrier(self):
        self.ctx._check(self.lib.tmpc_comm_barrier(self.h), "tmpc_comm_barrier")

    def broadcast_device(self, d_ptr, nbytes, root=0):
        self.ctx._check(self.lib.tmpc_comm_broadcast(self.h, d_ptr, int(nbytes), int(root)), "tmpc_comm_broadcast")

    def allgather_device(self, d_send, d_recv, nbytes_per_rank):
        self.ctx._check(self.lib.tmpc_comm_allgather(self.h, d_send, d_recv, int(nbytes_per_rank)),
                        "tmpc_comm_allgather")

    def broadcast(self, arr, root=0):
        """Host array (same shape / dtype on every rank) broadcast from root, returned."""
        arr = np.ascontiguousarray(arr)
        d = self.ctx.alloc(max(8, arr.nbytes))
        try:
            self.ctx.h2d(d, arr)
            self.broadcast_device(d, arr.nbytes, root)
            out = np.empty_like(arr)
            self.ctx.d2h(out, d)
        finally:
            self.ctx.free(d)
        return out

    def allgather(self, arr):
        """Host array per rank -> [world, *arr.shape] on every rank (rank order)."""
        arr = np.ascontiguousarray(arr)
        ds, dr = self.ctx.alloc(max(8, arr.nbytes)), self.ctx.alloc(max(8, arr.nbytes * self.world))
        try:
            self.ctx.h2d(ds, arr)
            self.allgather_device(ds, dr, arr.nbytes)
            out = np.empty((self.world,) + arr.shape, dtype=arr.dtype)
            self.ctx.d2h(out, dr)
        finally:
            self.ctx.free(ds)
            self.ctx.free(dr)
        return out

    def max(self, v: float) -> float:
        a = np.array([float(v)])
        d = self.ctx.alloc(8)
        try:
            self.ctx.h2d(d, a)
            self.ctx._check(self.lib.tmpc_comm_allreduce_max_f64(self.h, d, 1), "tmpc_comm_allreduce_max_f64")
            self.ctx.d2h(a, d)
        finally:
            self.ctx.free(d)
        return float(a[0])


_default_ctx = {}


def default_context(device: int = 0) -> Context:
    """Process-wide context per device (the Python plugin classes share it)."""
    ctx = _default_ctx.get(device)
    if ctx is None:
        ctx = Context(device)
        _default_ctx[device] = ctx
    return ctx
