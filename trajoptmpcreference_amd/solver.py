"""TrajoptMPCReference -- the reference's solver class
(TrajoptMPCReference.py:29-760) with the SQP hot path on the GPU.

``SQP(x, u, N, dt, METHOD, options)`` keeps the reference signature and
return tuple ``(x, u, exit_sqp, exit_soft, outer_iter, sqp_iter)`` and fills
``self.trace`` with one dict per SQP step (:555-569, :691-743).
``SQP_batch`` solves B independent problems in one call -- the batched form
the GPU is built for.  Invalid plugins/options raise instead of exit().
"""
import copy
import enum

import numpy as np

from . import _native, hooks
from ._options import NO_OPTIONS, fresh
from .constraint import TrajoptConstraint
from .cost import QuadraticCost, TrajoptCost, UrdfCost
from .plant import TrajoptPlant, URDFPlant


class SQPSolverMethods(enum.Enum):
    N = "N"
    S = "S"
    PCG_J = "PCG-J"
    PCG_BJ = "PCG-BJ"
    PCG_SS = "PCG-SS"


class MPCSolverMethods(enum.Enum):
    iLQR = "iLQR"
    QP_N = "QP-N"
    QP_S = "QP-S"
    QP_PCG_J = "QP-PCG-J"
    QP_PCG_BJ = "QP-PCG-BJ"
    QP_PCG_SS = "QP-PCG-SS"


# options['precision'] (a build option; the reference is fp64): include/tmpc.h TMPC_PRECISION_*
_PRECISION = {"fp64": 0, "fp32": 1, "mixed": 2}

_OPTION_MAP = {
    "exit_tolerance_linSys": "exit_tolerance_linSys",
    "max_iter_linSys": "max_iter_linSys",
    "exit_tolerance_SQP_DDP": "exit_tolerance_SQP_DDP",
    "max_iter_SQP_DDP": "max_iter_SQP_DDP",
    "alpha_factor_SQP_DDP": "alpha_factor_SQP_DDP",
    "alpha_min_SQP_DDP": "alpha_min_SQP_DDP",
    "rho_factor_SQP_DDP": "rho_factor_SQP_DDP",
    "rho_min_SQP_DDP": "rho_min_SQP_DDP",
    "rho_max_SQP_DDP": "rho_max_SQP_DDP",
    "rho_init_SQP_DDP": "rho_init_SQP_DDP",
    "expected_reduction_min_SQP_DDP": "expected_reduction_min_SQP_DDP",
    "expected_reduction_max_SQP_DDP": "expected_reduction_max_SQP_DDP",
    "max_iter_softConstraints": "max_iter_softConstraints",
    "exit_tolerance_softConstraints": "exit_tolerance_softConstraints",
}


def _method_name(m):
    if isinstance(m, SQPSolverMethods):
        return m.value
    if isinstance(m, str) and m in [e.value for e in SQPSolverMethods]:
        return m
    raise ValueError("Invalid QP Solver options are: N, S, PCG-J, PCG-BJ, PCG-SS")


class TrajoptMPCReference:
    def __init__(self, plantObj: TrajoptPlant, costObj: TrajoptCost, constraintObj: TrajoptConstraint = None):
        if not isinstance(plantObj, TrajoptPlant) or not isinstance(costObj, TrajoptCost):
            raise TypeError("Must pass in a TrajoptPlant and TrajoptCost object to TrajoptMPCReference.")
        if constraintObj is None:
            constraintObj = TrajoptConstraint()
        elif not isinstance(constraintObj, TrajoptConstraint):
            raise TypeError("If passing in additional constraints must pass in a TrajoptConstraint object.")
        self.plant = plantObj
        self.cost = costObj
        self.other_constraints = constraintObj
        self.trace = []
        self.n_inner_iter = 0
        self.exit_soft = 0
        self.exit_sqp = 0
        self.singular = False
        self.active_sets = []

    def update_cost(self, costObj: TrajoptCost):
        if not isinstance(costObj, TrajoptCost):
            raise TypeError("Must pass in a TrajoptCost object to update_cost in TrajoptMPCReference.")
        self.cost = costObj

    def update_plant(self, plantObj: TrajoptPlant):
        if not isinstance(plantObj, TrajoptPlant):
            raise TypeError("Must pass in a TrajoptPlant object to update_plant in TrajoptMPCReference.")
        self.plant = plantObj

    def update_constraints(self, constraintObj: TrajoptConstraint):
        if not isinstance(constraintObj, TrajoptConstraint):
            raise TypeError("Must pass in a TrajoptConstraint object to update_constraints in TrajoptMPCReference.")
        self.other_constraints = constraintObj

    def set_default_options(self, options: dict):
        """TrajoptMPCReference.py:91-115 (mutates the dict, as the reference does)."""
        options.setdefault("exit_tolerance_linSys", 1e-6)
        options.setdefault("max_iter_linSys", 100)
        options.setdefault("DEBUG_MODE_linSys", False)
        options.setdefault("RETURN_TRACE_linSys", False)
        # plant.rbdReference.overloading (:97); a plugin plant without an rbdReference does no tracing
        options.setdefault("overloading", getattr(getattr(self.plant, "rbdReference", None), "overloading", False))
        options.setdefault("exit_tolerance_SQP_DDP", 1e-6)
        options.setdefault("max_iter_SQP_DDP", 100)
        options.setdefault("DEBUG_MODE_SQP_DDP", False)
        options.setdefault("alpha_factor_SQP_DDP", 0.5)
        options.setdefault("alpha_min_SQP_DDP", 0.005)
        options.setdefault("rho_factor_SQP_DDP", 4)
        options.setdefault("rho_min_SQP_DDP", 1e-3)
        options.setdefault("rho_max_SQP_DDP", 1e3)
        options.setdefault("rho_init_SQP_DDP", 0.001)
        options.setdefault("expected_reduction_min_SQP_DDP", 0.05)
        options.setdefault("expected_reduction_max_SQP_DDP", 3)
        options.setdefault("merit_factor_SQP", 1.5)
        options.setdefault("exit_tolerance_softConstraints", 1e-6)
        options.setdefault("max_iter_softConstraints", 10)

    # ------------------------------------------------------------------ lowering to libtmpc
    def _check_xu(self, x, u, N):
        """x [B][nx][N], u [B][nu][N-1] with the plant's nx = 2 n, nu = n (the reference's
        column-per-knot arrays, TrajoptMPCReference.py:510, batched)."""
        nx, nu = self.plant.get_num_pos() + self.plant.get_num_vel(), self.plant.get_num_cntrl()
        if x.ndim != 3 or u.ndim != 3 or x.shape[0] != u.shape[0] or x.shape[1:] != (nx, N) \
                or u.shape[1:] != (nu, N - 1):
            raise ValueError(f"expected x [B][{nx}][{N}] and u [B][{nu}][{N - 1}], got {x.shape} and {u.shape}")

    def _hooks(self):
        """True when a plugin's hooks are the caller's own (a TrajoptCost / TrajoptPlant / TrajoptConstraint
        subclass, or one overriding a built-in's hooks): SQP then runs the plugin-hook path (hooks.py), the
        reference's loop over those hooks with every QP on the GPU.  The built-ins run wholly on the device."""
        return hooks.needs_hooks(self.plant, self.cost, self.other_constraints)

    def _hook_context(self, options):
        """A context for the plugin-hook path: only the linear-system options matter (the blocks come from
        the hooks)."""
        ctx = _native.default_context(getattr(self.plant, "device", 0))
        ctx.set_options(**{v: options[k] for k, v in _OPTION_MAP.items()})
        return ctx

    def _context(self, options):
        if self._hooks():
            which = [name for name, ok in (("cost", hooks.device_cost(self.cost) is not None),
                                           ("plant", hooks.device_plant(self.plant)),
                                           ("constraints", hooks.device_constraints(self.other_constraints)))
                     if not ok]
            raise NotImplementedError(
                f"this entry point runs on device plugins only; the {' / '.join(which)} hooks here are the "
                f"caller's own ({type(self.cost).__name__}, {type(self.plant).__name__}, "
                f"{type(self.other_constraints).__name__}): SQP / SQP_batch / solveKKTSystem(_Schur) honour them "
                f"(the plugin-hook path, hooks.py)")
        spec = self.other_constraints.gpu_spec()   # raises for ADMM_PROJECTION (the reference exits too)
        if options.get("overloading"):
            raise NotImplementedError("overloading (op-history tracing) is instrumentation, not offered")
        ctx = self.plant._ctx()
        c = self.cost
        if isinstance(c, UrdfCost):
            m = self.plant.model
            ctx.set_cost_ee(c.Q, c.QF, c.R, c.xg, c.QF_start, m.H0[:2], m.Ha[:2], m.Hb[:2])
        else:
            ctx.set_cost_quadratic(c.Q, c.QF, c.R, c.xg, c.QF_start)
        # pcg_warm_start (build option, default off = the reference): PCG of each QP starts from the
        # previous QP's lambda, across MPC steps from the shifted last lambda (include/tmpc.h)
        prec = options.get("precision", "fp64")
        if prec not in _PRECISION:
            raise ValueError(f"options['precision'] must be one of {sorted(_PRECISION)}, got {prec!r}")
        if prec != "fp64" and isinstance(c, UrdfCost):
            raise NotImplementedError("the fp32 / mixed precision modes support QuadraticCost only")
        ctx.set_options(**{v: options[k] for k, v in _OPTION_MAP.items()},
                        pcg_warm_start=int(bool(options.get("pcg_warm_start", False))), precision=_PRECISION[prec])
        ctx.set_box_limits(spec)
        return ctx

    def SQP_batch(self, x, u, N: int, dt: float, LINEAR_SYSTEM_SOLVER_METHOD=SQPSolverMethods.PCG_SS, options=None,
                  soft_state=None, hard_active=False):
        """B problems at once: x [B][nx][N], u [B][nu][N-1] -> dict of per-problem results.
        With soft limits every problem starts from the constraint objects' mu / lambda / phi
        (or from soft_state = (mu, lam, phi), each [B][N][6n]); the final per-problem
        constants are returned as r["soft_state"].  hard_active: with hard limits, also every QP's
        active set (r["trace"]["hard_active"] [B][max_iter+1][N] bitmasks, include/tmpc.h)."""
        options = {} if options is None else options
        self.set_default_options(options)
        # method N (solveKKTSystem, the dense KKT solve, :313-359) has the Schur complement's solution and
        # runs the direct Schur path with the same least-squares fallback (include/tmpc.h TMPC_LINSYS_N)
        method = _method_name(LINEAR_SYSTEM_SOLVER_METHOD)
        if self._hooks():
            return self._sqp_hooks_batch(x, u, N, dt, method, options, soft_state)
        ctx = self._context(options)
        x = np.asarray(x, dtype=np.float64)
        u = np.asarray(u, dtype=np.float64)
        self._check_xu(x, u, N)
        B = x.shape[0]
        soft = self.other_constraints.has_any()
        if soft:
            if self.other_constraints.num_timesteps != N:
                raise ValueError(f"TrajoptConstraint was built for {self.other_constraints.num_timesteps} knots, "
                                 f"solving with N = {N}")
            if soft_state is None:
                soft_state = [np.broadcast_to(a, (B,) + a.shape) for a in self.other_constraints.pack_state(N)]
            ctx.set_soft_state(B, N, *soft_state)
        r = ctx.sqp_solve_batch(x, u, N, dt, method, hard_active=hard_active)
        if soft:
            r["soft_state"] = ctx.get_soft_state(B, N)
        return r

    def _sqp_hooks_batch(self, x, u, N, dt, method, options, soft_state):
        """SQP_batch on the plugin-hook path (hooks.py).  Every problem runs on its own copy of the constraint
        object (the device path's per-problem soft state), so the caller's object is left unchanged and a
        repeated call gives the same results; with soft limits r["soft_state"] holds every problem's final
        constants (SQP() writes them back through unpack_state, as on the device path)."""
        if options.get("overloading"):
            raise NotImplementedError("overloading (op-history tracing) is instrumentation, not offered")
        x = np.asarray(x, dtype=np.float64)
        u = np.asarray(u, dtype=np.float64)
        self._check_xu(x, u, N)
        B = x.shape[0]
        ctx = self._hook_context(options)
        con = self.other_constraints
        soft = con.has_any()
        if soft and con.num_timesteps != N:
            raise ValueError(f"TrajoptConstraint was built for {con.num_timesteps} knots, solving with N = {N}")
        outs, states = [], []
        try:
            for b in range(B):
                self.other_constraints = copy.deepcopy(con)
                if soft and soft_state is not None:
                    self.other_constraints.unpack_state(*[np.asarray(a)[b] for a in soft_state])
                outs.append(hooks.sqp_hooks_batch(self, ctx, x[b:b + 1], u[b:b + 1], N, dt, method, options))
                if soft:
                    states.append(self.other_constraints.pack_state(N))
        finally:
            self.other_constraints = con
        r = {k: np.concatenate([o[k] for o in outs]) for k in ("exit_sqp", "exit_soft", "outer_iter", "sqp_iter",
                                                                "x", "u")}
        r["trace"] = {k: np.concatenate([o["trace"][k] for o in outs]) for k in outs[0]["trace"]}
        if soft:
            r["soft_state"] = tuple(np.array([st[i] for st in states]) for i in range(3))
        return r

    def SQP(self, x, u, N: int, dt: float, LINEAR_SYSTEM_SOLVER_METHOD=SQPSolverMethods.N, options=NO_OPTIONS):
        """TrajoptMPCReference.SQP (:510-760) for one problem."""
        options = fresh(options)
        x = np.asarray(x, dtype=np.float64)
        u = np.asarray(u, dtype=np.float64)
        hard = any(c.is_hard_constraint_mode() for _, c in self.other_constraints.limits())
        r = self.SQP_batch(x[None], u[None], N, dt, LINEAR_SYSTEM_SOLVER_METHOD, options, hard_active=hard)
        method = _method_name(LINEAR_SYSTEM_SOLVER_METHOD)
        it = int(r["sqp_iter"][0])
        t = r["trace"]
        # one row per SQP iteration run plus the initial row; the iteration counter is not
        # incremented by the max_iter exit (check_for_exit_or_error :475-479)
        rows = min(it + 1 + (int(r["exit_sqp"][0]) == 3), t["alpha"].shape[1])
        # the trace is that of the last outer pass, whose index is outer_iter unless the outer
        # loop exited with code 1 or 3 (which increment the counter first, :490-499)
        ex_soft, outer = int(r["exit_soft"][0]), int(r["outer_iter"][0])
        last_pass = outer if ex_soft == 2 else outer - 1
        if "soft_state" in r:
            self.other_constraints.unpack_state(*[a[0] for a in r["soft_state"]])
        # self.singular is sticky over the object's life, as the reference's (:74, :356, :435)
        sing_rows = [bool(v) for v in t["singular"][0, :rows]]
        self.trace = []
        for i in range(rows):
            if i:
                self.singular = self.singular or sing_rows[i]
            self.trace.append({
                "outer_iteration": last_pass,
                "iteration": int(t["iteration"][0, i]),
                "line_search_iteration": int(t["line_search_iteration"][0, i]),
                "alpha": float(t["alpha"][0, i]) if i else 1,
                "rho": float(t["rho"][0, i]),
                "J": float(t["J"][0, i]),
                "c": float(t["c"][0, i]),
                "merit": float(t["merit"][0, i]),
                "D": None if i == 0 else float(t["D"][0, i]),
                "reduction_ratio": None if i == 0 else float(t["reduction_ratio"][0, i]),
                # the true PCG iteration count (the reference stores len((trace, trace2)) == 2: SURVEY F7)
                "inner_iters": int(t["pcg_iters"][0, i]) if method.startswith("PCG") else 0,
                "singular": self.singular if i else False,
                "succeeded_line_search": bool(t["succeeded_line_search"][0, i]),
            })
        # with hard limits: each QP's active set, per knot a bitmask (bit t * 2n + e; include/tmpc.h) --
        # the rows the reference appends to C (TrajoptMPCReference.py:238-248), one list per trace row
        self.active_sets = [[int(v) for v in t["hard_active"][0, i]] for i in range(1, rows)] if hard else []
        self.exit_sqp = int(r["exit_sqp"][0])
        self.exit_soft = int(r["exit_soft"][0])
        return (r["x"][0], r["u"][0], self.exit_sqp, self.exit_soft, int(r["outer_iter"][0]), it)

    # ------------------------------------------------------------------ iLQR (MPCSolverMethods.iLQR)
    def iLQR_batch(self, x, u, N: int, dt: float, options=None, soft_state=None):
        """Batched iLQR (algorithm in oracle/ilqr.py -- the reference defines only
        the MPCSolverMethods.iLQR enum value).  Same plugins, *_SQP_DDP options, rho schedule, exit
        codes and soft-constraint outer loop as SQP_batch; x is replaced by the rollout of u from
        x[:, :, 0]."""
        options = {} if options is None else options
        self.set_default_options(options)
        ctx = self._context(options)
        x = np.asarray(x, dtype=np.float64)
        u = np.asarray(u, dtype=np.float64)
        self._check_xu(x, u, N)
        B = x.shape[0]
        soft = self.other_constraints.has_any()
        if soft:
            if soft_state is None:
                soft_state = [np.broadcast_to(a, (B,) + a.shape) for a in self.other_constraints.pack_state(N)]
            ctx.set_soft_state(B, N, *soft_state)
        r = ctx.ilqr_solve_batch(x, u, N, dt)
        if soft:
            r["soft_state"] = ctx.get_soft_state(B, N)
        return r

    def iLQR(self, x, u, N: int, dt: float, options=None):
        """One problem: returns (x, u, exit_code, exit_soft, outer_iter, iter) like SQP, trace in self.trace."""
        r = self.iLQR_batch(np.asarray(x, dtype=np.float64)[None], np.asarray(u, dtype=np.float64)[None], N, dt,
                            options)
        it = int(r["iter"][0])
        t = r["trace"]
        ex_soft, outer = int(r["exit_soft"][0]), int(r["outer_iter"][0])
        last_pass = outer if ex_soft == 2 else outer - 1
        if "soft_state" in r:
            self.other_constraints.unpack_state(*[a[0] for a in r["soft_state"]])
        self.trace = []
        for i in range(min(it + 1 + (int(r["exit_code"][0]) == 3), t["alpha"].shape[1])):
            self.trace.append({
                "outer_iteration": last_pass,
                "iteration": int(t["iteration"][0, i]),
                "line_search_iteration": int(t["line_search_iteration"][0, i]),
                "alpha": float(t["alpha"][0, i]) if i else 1,
                "rho": float(t["rho"][0, i]),
                "J": float(t["J"][0, i]),
                "dV1": None if i == 0 or np.isnan(t["D"][0, i]) else float(t["D"][0, i]),
                "reduction_ratio": None if i == 0 or np.isnan(t["reduction_ratio"][0, i])
                else float(t["reduction_ratio"][0, i]),
                "succeeded_line_search": bool(t["succeeded_line_search"][0, i]),
            })
        self.exit_sqp = int(r["exit_code"][0])
        self.exit_soft = ex_soft
        return (r["x"][0], r["u"][0], self.exit_sqp, self.exit_soft, outer, it)

    # ------------------------------------------------------------------ receding-horizon MPC
    def MPC_batch(self, x, u, N: int, dt: float, SOLVER_METHOD=MPCSolverMethods.QP_PCG_SS, options=None,
                  mpc_steps: int = 1, soft_state=None):
        """Receding-horizon loop for B problems (algorithm in oracle/mpc.py -- the
        reference calls runMPCExample but never defines it, F1).  Each step solves the horizon with
        SQP (QP-S / QP-PCG-*) or iLQR warm-started from the shifted previous solution, applies u[:, 0]
        for one Euler step and shifts; the cost's QF_start and the soft-limit constants shift as the
        reference's hooks do (TrajoptCost.py:100-104, TrajoptConstraint.py:168-176).  Returns the
        executed states [B][nx][steps+1] / controls [B][nu][steps] and per-step exit codes / iterations."""
        options = {} if options is None else options
        self.set_default_options(options)
        m = SOLVER_METHOD.value if isinstance(SOLVER_METHOD, MPCSolverMethods) else str(SOLVER_METHOD)
        if m == "iLQR":
            solver = "iLQR"
        elif m.startswith("QP-") and m[3:] in ("N", "S", "PCG-J", "PCG-BJ", "PCG-SS"):
            solver = m[3:]   # QP-N: the dense KKT solve, the Schur complement's solution (method N of SQP)
        else:
            raise NotImplementedError(f"MPC solver {m}: use iLQR, QP-N, QP-S, QP-PCG-J, QP-PCG-BJ or QP-PCG-SS")
        ctx = self._context(options)
        x = np.asarray(x, dtype=np.float64)
        u = np.asarray(u, dtype=np.float64)
        self._check_xu(x, u, N)
        B = x.shape[0]
        soft = self.other_constraints.has_any()
        if soft:
            if soft_state is None:
                soft_state = [np.broadcast_to(a, (B,) + a.shape) for a in self.other_constraints.pack_state(N)]
            ctx.set_soft_state(B, N, *soft_state)
        r = ctx.mpc_batch(x, u, N, dt, solver, int(mpc_steps))
        if soft:
            r["soft_state"] = ctx.get_soft_state(B, N)
        if self.cost.QF_start is not None:
            self.cost.QF_start = max(self.cost.QF_start - int(mpc_steps), 0)
        return r

    def MPC(self, x, u, N: int, dt: float, SOLVER_METHOD=MPCSolverMethods.QP_PCG_SS, options=None, mpc_steps: int = 1):
        """One problem: returns (x_exec [nx][steps+1], u_exec [nu][steps], exit_codes, iters)."""
        r = self.MPC_batch(np.asarray(x, dtype=np.float64)[None], np.asarray(u, dtype=np.float64)[None], N, dt,
                           SOLVER_METHOD, options, mpc_steps)
        if "soft_state" in r:
            self.other_constraints.unpack_state(*[a[0] for a in r["soft_state"]])
        return r["x_exec"][0], r["u_exec"][0], r["exit_codes"][0], r["iters"][0]

    # ------------------------------------------------------------------ the reference's QP-level methods
    # formKKTSystemBlocks / solveKKTSystem / solveKKTSystem_Schur / totalCost / totalHardConstraintViolation /
    # reduce_regularization / check_for_exit_or_error / check_and_update_soft_constraints
    # (TrajoptMPCReference.py:118-508) for callers that drive the SQP steps themselves.  The dynamics and the
    # QP solve run on the GPU (tmpc_fd_batch / tmpc_fd_grad_batch / tmpc_qp_batch); the dense matrices these
    # methods return are assembled from the device's blocks at this boundary, in the reference's layout.
    def _dims(self):
        nq, nv, nu = self.plant.get_num_pos(), self.plant.get_num_vel(), self.plant.get_num_cntrl()
        return nq + nv, nu

    def _dynamics(self, x, u, N, dt, return_gradient=False):
        """The integrator over knots 0..N-2 (TrajoptPlant.integrator, :83-108): one GPU launch for a plant
        with device dynamics, else the plant's own hook knot by knot (the plugin-hook path)."""
        X, U = x[:, :N - 1].T, u[:, :N - 1].T
        if hooks.device_plant(self.plant):
            return self.plant.integrator_batch(X, U, dt, return_gradient=return_gradient)
        r = [self.plant.integrator(x[:, k], u[:, k], dt, return_gradient=return_gradient) for k in range(N - 1)]
        if return_gradient:
            return np.array([a for a, _ in r]), np.array([b for _, b in r])
        return np.array(r)

    def formKKTSystemBlocks(self, x, u, xs, N: int, dt: float):
        """formKKTSystemBlocks (:118-271, the NumPy branch :200-271): dense G, g, C, c of the QP at (x, u).
        A_k, B_k and f(x_k, u_k) of all N - 1 knots come from one GPU launch each; cost hessian / gradient,
        the soft-limit jacobian terms (:220-225, :255-259) and the hard-limit rows appended after each
        knot's dynamics rows (:238-248, :262-270) are the plugins' own hooks, placed as the reference
        places them."""
        self._check_reference_hooks()
        nx, nu = self._dims()
        n = nx + nu
        x = np.asarray(x, dtype=np.float64)
        u = np.asarray(u, dtype=np.float64)
        xs = np.asarray(xs, dtype=np.float64).reshape(-1)
        A, B = self._dynamics(x, u, N, dt, return_gradient=True)
        xkp1 = self._dynamics(x, u, N, dt)
        con = self.other_constraints
        nz = n * (N - 1) + nx
        n_other = con.total_hard_constraints(x, u)
        G = np.zeros((nz, nz))
        g = np.zeros((nz, 1))
        C = np.zeros((nx * N + n_other, nz))
        c = np.zeros((nx * N + n_other, 1))
        ci, si = 0, 0
        C[ci:ci + nx, si:si + nx] = np.eye(nx)
        c[ci:ci + nx, 0] = x[:, 0] - xs
        ci += nx
        for k in range(N - 1):
            G[si:si + n, si:si + n] = self.cost.hessian(x[:, k], u[:, k], k)
            g[si:si + n, 0] = self.cost.gradient(x[:, k], u[:, k], k)
            if con.total_soft_constraints(timestep=k) > 0:
                gck = con.jacobian_soft_constraints(x[:, k], u[:, k], k)
                g[si:si + n, :] = g[si:si + n, :] + gck
                G[si:si + n, si:si + n] += hooks.soft_hessian(con, x[:, k], u[:, k], k, np.ravel(gck))
            C[ci:ci + nx, si:si + n + nx] = np.hstack((-A[k], -B[k], np.eye(nx)))
            c[ci:ci + nx, 0] = x[:, k + 1] - xkp1[k]
            ci += nx
            if n_other > 0 and con.total_hard_constraints(x, u, k):
                jac = con.jacobian_hard_constraints(x[:, k], u[:, k], k)
                val = con.value_hard_constraints(x[:, k], u[:, k], k)
                if val is not None and len(val):
                    m = len(val)
                    C[ci:ci + m, si:si + n] = np.reshape(jac, (m, n))
                    c[ci:ci + m] = np.reshape(val, (m, 1))
                    ci += m
            si += n
        G[si:si + nx, si:si + nx] = self.cost.hessian(x[:, N - 1], timestep=N - 1)
        g[si:si + nx, 0] = self.cost.gradient(x[:, N - 1], timestep=N - 1)
        if con.total_soft_constraints(timestep=N - 1) > 0:
            # the terminal knot has only x: the state part of the column (oracle/soft.py; the reference adds
            # an n_xu column to an nx slice there)
            gc = np.ravel(con.jacobian_soft_constraints(x[:, N - 1], timestep=N - 1))[:nx]
            g[si:si + nx, 0] = g[si:si + nx, 0] + gc
            G[si:si + nx, si:si + nx] = G[si:si + nx, si:si + nx] + \
                hooks.soft_hessian(con, x[:, N - 1], None, N - 1, gc)[:nx, :nx]
        if n_other > 0 and con.total_hard_constraints(x, u, N - 1):
            jac = con.jacobian_hard_constraints(x[:, N - 1], timestep=N - 1)
            val = con.value_hard_constraints(x[:, N - 1], timestep=N - 1)
            if val is not None and len(val):
                m = len(val)
                C[ci:ci + m, si:si + nx] = np.reshape(jac, (m, nx))
                c[ci:ci + m] = np.reshape(val, (m, 1))
        return G, g, C, c

    def totalHardConstraintViolation(self, x, u, xs, N: int, dt: float, mode=None):
        """totalHardConstraintViolation (:273-294): |x_0 - xs|_1 + sum_k |x_{k+1} - f(x_k, u_k)|_1 (+ the hard
        limits' |values|), each term summed as the reference sums it; mode "MAX" takes max instead of sum.
        f of all knots is one GPU launch."""
        mode_func = max if mode == "MAX" else sum
        x = np.asarray(x, dtype=np.float64)
        u = np.asarray(u, dtype=np.float64)
        xs = np.asarray(xs, dtype=np.float64).reshape(-1)
        xkp1 = self._dynamics(x, u, N, dt)
        c = mode_func(list(map(abs, x[:, 0] - xs)))
        for k in range(N - 1):
            c = c + mode_func(list(map(abs, x[:, k + 1] - xkp1[k])))
        con = self.other_constraints
        if con.total_hard_constraints(x, u) > 0:
            for k in range(N - 1):
                if con.total_hard_constraints(x, u, k):
                    c = c + mode_func(list(map(abs, con.value_hard_constraints(x[:, k], u[:, k], k))))
            if con.total_hard_constraints(x, u, N - 1):
                # the reference passes N - 1 as uk here (:292), which value_hard_constraints then ignores for
                # the terminal knot's state limits
                c = c + mode_func(list(map(abs, con.value_hard_constraints(x[:, N - 1], timestep=N - 1))))
        return c

    def totalCost(self, x, u, N: int):
        """totalCost (:296-310): sum of the cost hook over the knots (terminal: u = None), plus the soft
        limits' values, in the reference's order."""
        x = np.asarray(x, dtype=np.float64)
        u = np.asarray(u, dtype=np.float64)
        J = 0
        for k in range(N - 1):
            J = J + self.cost.value(x[:, k], u[:, k], k)
        J = J + self.cost.value(x[:, N - 1], timestep=N - 1)
        con = self.other_constraints
        if con.total_soft_constraints() > 0:
            for k in range(N - 1):
                J = J + con.value_soft_constraints(x[:, k], u[:, k], k)
            J = J + con.value_soft_constraints(x[:, N - 1], timestep=N - 1)
        return J

    def _check_reference_hooks(self):
        """With reference_hooks the constraint hooks are the reference's (velocity limits on q, vstacked
        jacobians): for soft velocity limits or several soft kinds they describe a QP that neither the
        device nor the reference's own SQP can form, so the QP-level methods refuse them."""
        con = self.other_constraints
        if not getattr(con, "reference_hooks", False):
            return
        soft = [k for k, c in con.limits() if c.is_soft_constraint_mode()]
        if "velocity_limits" in soft or len(soft) > 1:
            raise NotImplementedError("reference_hooks with soft velocity limits or several soft limit kinds: "
                                      "the reference's hooks read q for velocity limits and vstack the kinds' "
                                      "jacobians, which no QP consumes (SURVEY F6); unset reference_hooks")

    def _qp(self, x, u, xs, N, dt, rho, method, options):
        """One QP on the GPU (tmpc_qp_batch) -> the reference's dxul column [dxu; lambda], lambda in the
        reference's row order (initial state, then per knot its dynamics rows and its active hard rows).
        options are the reference's linear-system options (solveKKTSystem_Schur passes PCG's keys:
        exit_tolerance, max_iter, preconditioner_type, guess -- PCG.py:19-25, :439-440); the caller's dict
        is not modified."""
        self._check_reference_hooks()
        opts = dict(options)
        self.set_default_options(opts)
        if "exit_tolerance" in opts:
            opts["exit_tolerance_linSys"] = opts["exit_tolerance"]
        if "max_iter" in opts:
            opts["max_iter_linSys"] = opts["max_iter"]
        nx, nu = self._dims()
        x = np.asarray(x, dtype=np.float64)
        u = np.asarray(u, dtype=np.float64)
        xs = np.asarray(xs, dtype=np.float64).reshape(1, -1)
        self._check_xu(x[None], u[None], N)
        guess = opts.get("guess") if method.startswith("PCG") else None
        if guess is not None:   # options['guess'] -> PCG.update_guess (:439-440)
            guess = np.asarray(guess, dtype=np.float64).reshape(1, -1)
            if guess.shape[1] != N * nx:
                raise ValueError(f"options['guess'] must have N * nx = {N * nx} entries, got {guess.shape[1]}")
        if self._hooks():   # the plugin-hook path: the hooks form the blocks, the GPU solves the QP
            if any(c.is_hard_constraint_mode() for _, c in self.other_constraints.limits()):
                raise NotImplementedError("hard box constraints with plugin-hook costs or plants (hooks.py)")
            hs = hooks._HookSQP(self, self._hook_context(opts), N, dt, method, opts)
            G, g, A, Bm, c = hs.blocks(x, u, xs[0])
            r = hs.ctx.qp_blocks_batch(G[None], g[None], A[None], Bm[None], c[None], rho, method, guess=guess)
            self.n_inner_iter = int(r["pcg_iters"][0])
            return r["dxul"][0].reshape(-1, 1)
        ctx = self._context(opts)
        con = self.other_constraints
        if any(c.is_soft_constraint_mode() for _, c in con.limits()):   # the objects' current mu / lambda
            ctx.set_soft_state(1, N, *[a[None] for a in con.pack_state(N)])
        r = ctx.qp_batch(x[None], u[None], N, dt, rho, method, want_blocks=False, guess=guess, xs=xs)
        self.n_inner_iter = int(r["pcg_iters"][0])
        dxul = r["dxul"][0]
        if not any(c.is_hard_constraint_mode() for _, c in con.limits()):
            return dxul.reshape(-1, 1)
        info = ctx.qp_hard_info(1, N)
        if int(info["singular"][0]):
            self.singular = True
        nz = (nx + nu) * (N - 1) + nx
        lam_dyn = dxul[nz:].reshape(N, nx)
        lam_h = info["lambda_hard"][0]
        n = nx // 2
        lam = [lam_dyn[0]]
        for k in range(N):
            if k < N - 1:
                lam.append(lam_dyn[k + 1])
            slots = []
            for kind, cobj, z in con._hard_slices(x[:, k], u[:, k] if k < N - 1 else None,
                                                  k if k < N - 1 else N - 1):
                t = {"joint_limits": 0, "velocity_limits": 1, "torque_limits": 2}[kind]
                v = cobj.full_value(z)
                for e in range(2 * cobj.constraint_size):
                    if cobj.mode == "FULL_SET" or v[e] < 0:
                        slots.append(t * 2 * n + e)
            lam.append(lam_h[k, slots])
        return np.concatenate([dxul[:nz]] + lam).reshape(-1, 1)

    def solveKKTSystem(self, x, u, xs, N: int, dt: float, rho: float = 0.0, options=NO_OPTIONS):
        """solveKKTSystem (:313-359): the dense KKT [G + rho I, C^T; C, 0] dxul = [g; c].  Its solution is
        the Schur complement's, so the GPU solves it blockwise by the direct path (method N: block-Thomas,
        or the banded elimination with hard limits) with the reference's least-squares fallback for a
        singular system (self.singular)."""
        return self._qp(x, u, xs, N, dt, rho, "N", fresh(options))

    def solveKKTSystem_Schur(self, x, u, xs, N: int, dt: float, rho: float = 0.0, use_PCG=False, options=NO_OPTIONS):
        """solveKKTSystem_Schur (:361-455): S = -C G^-1 C^T, gamma = c - C G^-1 g, lambda by the direct solve
        (use_PCG False, the reference's default) or PCG with options['preconditioner_type'] (default BJ,
        PCG.py:24) and options['guess'] as the initial iterate; dxu = G^-1 (g - C^T lambda)."""
        options = fresh(options)
        method = "PCG-" + options.get("preconditioner_type", "BJ") if use_PCG else "S"
        return self._qp(x, u, xs, N, dt, rho, method, options)

    def reduce_regularization(self, rho: float, drho: float, options: dict):
        """reduce_regularization (:457-461)."""
        self.set_default_options(options)
        drho = min(drho / options["rho_factor_SQP_DDP"], 1 / options["rho_factor_SQP_DDP"])
        rho = max(rho * drho, options["rho_min_SQP_DDP"])
        return rho, drho

    def check_for_exit_or_error(self, error: bool, delta_J: float, iteration: int, rho: float, drho: float, options):
        """check_for_exit_or_error (:463-481): the error branch raises rho (exit 2 past rho_max), a cost
        decrease below the tolerance exits 1 (signed: any increase exits too), the last iteration exits 3."""
        self.set_default_options(options)
        exit_flag = False
        if error:
            drho = max(drho * options["rho_factor_SQP_DDP"], options["rho_factor_SQP_DDP"])
            rho = max(rho * drho, options["rho_min_SQP_DDP"])
            if rho > options["rho_max_SQP_DDP"]:
                self.exit_sqp = 2
                exit_flag = True
        elif delta_J < options["exit_tolerance_SQP_DDP"]:
            self.exit_sqp = 1
            exit_flag = True
        if iteration == options["max_iter_SQP_DDP"] - 1:
            self.exit_sqp = 3
            exit_flag = True
        else:
            iteration += 1
        return exit_flag, iteration, rho, drho

    def check_and_update_soft_constraints(self, x, u, iteration: int, options):
        """check_and_update_soft_constraints (:483-508): exit_soft 1 (converged), 2 (max outer passes),
        3 (every violated mu at its cap), else the AL update of the constraint objects' constants."""
        exit_flag = False
        if self.other_constraints.max_soft_constraint_value(x, u) < options["exit_tolerance_softConstraints"]:
            self.exit_soft = 1
            exit_flag = True
        if iteration == options["max_iter_softConstraints"] - 1:
            self.exit_soft = 2
            exit_flag = True
        else:
            iteration += 1
        if not exit_flag:
            if self.other_constraints.update_soft_constraint_constants(x, u):
                self.exit_soft = 3
                exit_flag = True
        return exit_flag, iteration
