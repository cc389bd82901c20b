"""The plugin-hook path of the drop-in: TrajoptMPCReference.SQP (TrajoptMPCReference.py:510-760) driven
on the host over the caller's own TrajoptCost / TrajoptPlant / TrajoptConstraint hooks, with the QP on
the GPU.

The built-in plugins (QuadraticCost, UrdfCost, URDFPlant, the box limits) have device implementations and
the whole SQP runs on the device (csrc/tmpc_api.cpp sqp_device).  A subclass that overrides one of their
hooks -- or any other TrajoptCost / TrajoptPlant subclass -- has none: its hooks are Python.  For those
the reference's own loop runs here, calling the hooks exactly where the reference calls them
(formKKTSystemBlocks :200-271, totalCost :296-310, totalHardConstraintViolation :273-294, the line-search
directional derivative :635-648) with the reference's iter_1 / iter_2 / iter_3 arguments, and every QP
-- (G + rho I)^-1, the Schur complement, PCG / the direct solve, dxu -- runs on the GPU on the blocks the
hooks formed (tmpc_qp_blocks_batch, csrc/tmpc_hooks.hip).  The dynamics stay on the GPU too whenever the
plant is a URDFPlant whose dynamics hooks are not overridden (one batched launch per knot sweep).
There is no CPU fallback for the QP: without the library the solve raises.

Supported: methods N, S, PCG-J / BJ / SS; soft constraints (QUADRATIC_PENALTY / AUGMENTED_LAGRANGIAN and
the outer loop, :483-508) through the constraint object's hooks; hard box constraints (ACTIVE_SET / FULL_SET,
:238-248): the constraint hooks' rows (value_hard_constraints / jacobian_hard_constraints) go to the banded
device QP with the plugin's blocks (tmpc_qp_blocks_banded_batch), which also takes QPs past the fused
kernel's 1024 rows.  A hard row must be a box row (one +-1 entry of [x_k; u_k], or a zero FULL_SET row),
as the reference's BoxConstraint produces; nx must be 2 nu.
"""
import copy

import numpy as np

from .constraint import TrajoptConstraint
from .cost import QuadraticCost, TrajoptCost, UrdfCost
from .plant import TrajoptPlant, URDFPlant

COST_HOOKS = ("value", "gradient", "hessian", "get_currQ", "delta_x", "jacobian_tot_state", "compute_J", "_kin")
PLANT_HOOKS = ("integrator", "forward_dynamics", "forward_dynamics_gradient", "qdd_to_xdot", "dqdd_to_dxdot",
               "integrator_batch", "forward_dynamics_batch", "forward_dynamics_gradient_batch", "minv_batch")
CONSTRAINT_HOOKS = ("total_soft_constraints", "value_soft_constraints", "jacobian_soft_constraints",
                    "max_soft_constraint_value", "update_soft_constraint_constants", "total_hard_constraints",
                    "value_hard_constraints", "jacobian_hard_constraints", "shift_soft_constraint_constants",
                    "_soft_slices", "_hard_slices")


def overrides(obj, base, names):
    """The hook names of `names` that type(obj) defines differently from `base` (a subclass's own override
    anywhere between type(obj) and base)."""
    t = type(obj)
    return [m for m in names if getattr(t, m, None) is not getattr(base, m, None)]


def device_cost(cost):
    """The cost the device evaluates, or None when its hooks are the caller's: QuadraticCost / UrdfCost
    themselves, or a subclass that overrides none of their hooks."""
    if not isinstance(cost, QuadraticCost):
        return None
    base = UrdfCost if isinstance(cost, UrdfCost) else QuadraticCost
    return None if overrides(cost, base, COST_HOOKS) else cost


def device_plant(plant):
    """True when the plant's dynamics are the device's: a URDFPlant (PendulumPlant included) whose
    dynamics hooks are not overridden."""
    if not isinstance(plant, URDFPlant):
        return False
    from .plant import PendulumPlant
    base = PendulumPlant if isinstance(plant, PendulumPlant) else URDFPlant
    return not overrides(plant, base, PLANT_HOOKS)


def device_constraints(con):
    return type(con) is TrajoptConstraint or not overrides(con, TrajoptConstraint, CONSTRAINT_HOOKS)


def soft_hessian(con, xk, uk, k, gck):
    """The soft limits' Hessian term of a knot: outer(jac, jac) of the caller's jacobian column, as the
    reference forms it (:223-225, :258-259), unless the jacobian hook is this package's own -- then the sum of
    the per-kind outer products (TrajoptConstraint.soft_outer), the device QP's term, which equals
    outer(jac, jac) for one soft kind."""
    if (isinstance(con, TrajoptConstraint) and not con.reference_hooks
            and not overrides(con, TrajoptConstraint, ("jacobian_soft_constraints", "_soft_slices"))):
        return con.soft_outer(xk, uk, k)
    return np.outer(gck, gck)


def needs_hooks(plant, cost, con):
    return device_cost(cost) is None or not device_plant(plant) or not device_constraints(con)


class _HookSQP:
    """One problem's SQP over the solver's plugin hooks (TrajoptMPCReference.SQP :510-760)."""

    def __init__(self, solver, ctx, N, dt, method, o):
        self.s, self.ctx, self.N, self.dt, self.method, self.o = solver, ctx, N, dt, method, o
        p = solver.plant
        self.nx = p.get_num_pos() + p.get_num_vel()
        self.nu = p.get_num_cntrl()
        self.n = self.nx + self.nu
        self.gpu_dyn = device_plant(p)
        self.it = self.outer = self.ls = 0
        con = solver.other_constraints
        # hard rows: the built-in box limits in a hard mode, or a subclass's own hard-constraint hooks
        self.hard = any(c.is_hard_constraint_mode() for _, c in con.limits()) or bool(
            overrides(con, TrajoptConstraint, ("total_hard_constraints", "value_hard_constraints",
                                               "jacobian_hard_constraints", "_hard_slices")))
        # the banded device QP: hard rows, or past the fused kernel's 1024 Schur rows
        self.banded = self.hard or N * self.nx > 1024
        self.mask = np.zeros(N, dtype=np.uint64)   # the last QP's active set per knot (trace hard_active)
        self.singular = 0

    # -- plugin evaluations, placed and called as the reference places and calls them.  The iter_* arguments
    # are the reference's module-global counters (overloading.matrix_): the initial cost / violation of an
    # outer pass sees the previous pass's final iteration and line-search indices (matrix_.iteration is reset
    # after them, :541-572), formKKTSystemBlocks sees the previous line search's last index (it is reset after
    # the QP, :608) and calls the integrator without iter_3 (:230-232); totalHardConstraintViolation passes
    # iter_3 (:282).  A fresh solve starts from 0, the globals' value at import.
    def _step(self, x, u, grad):
        """f(x_k, u_k) of all knots [N-1][nx]; with grad (formKKTSystemBlocks) also A [N-1][nx][nx],
        B [N-1][nx][nu], and the integrator called without iter_3 as there."""
        N, p = self.N, self.s.plant
        X, U = x[:, :N - 1].T, u[:, :N - 1].T
        if self.gpu_dyn:
            f = p.integrator_batch(X, U, self.dt)
            return (f,) + (p.integrator_batch(X, U, self.dt, return_gradient=True) if grad else ())
        kw = dict(iter_1=self.it, iter_2=self.outer) if grad else dict(iter_1=self.it, iter_2=self.outer,
                                                                         iter_3=self.ls)
        f = np.array([p.integrator(x[:, k], u[:, k], self.dt, **kw) for k in range(N - 1)])
        if not grad:
            return (f,)
        AB = [p.integrator(x[:, k], u[:, k], self.dt, return_gradient=True, iter_1=self.it, iter_2=self.outer)
              for k in range(N - 1)]
        return f, np.array([a for a, _ in AB]), np.array([b for _, b in AB])

    def total_cost(self, x, u):
        """totalCost (:296-310)"""
        N, cost, con = self.N, self.s.cost, self.s.other_constraints
        J = 0
        for k in range(N - 1):
            J = J + cost.value(x[:, k], u[:, k], k, self.it, self.outer, iter_3=self.ls)
        J = J + cost.value(x[:, N - 1], timestep=N - 1, iter_1=self.it, iter_2=self.outer, iter_3=self.ls)
        if con.total_soft_constraints() > 0:
            for k in range(N - 1):
                J = J + con.value_soft_constraints(x[:, k], u[:, k], k)
            J = J + con.value_soft_constraints(x[:, N - 1], timestep=N - 1)
        return J

    def violation(self, x, u, xs):
        """totalHardConstraintViolation (:273-294): the initial-state and dynamics defects' 1-norms knot by
        knot, then the hard constraints' (:286-293; the terminal value_hard_constraints call passes N - 1 in
        the u position, as the reference's)."""
        (f,) = self._step(x, u, False)
        c = sum(map(abs, x[:, 0] - xs))
        N = self.N
        for k in range(N - 1):
            c = c + sum(map(abs, x[:, k + 1] - f[k]))
        if self.hard:
            con = self.s.other_constraints
            if con.total_hard_constraints(x, u) > 0:
                for k in range(N - 1):
                    if con.total_hard_constraints(x, u, k):
                        c = c + sum(map(abs, con.value_hard_constraints(x[:, k], u[:, k], k)))
                if con.total_hard_constraints(x, u, N - 1):
                    c = c + sum(map(abs, con.value_hard_constraints(x[:, N - 1], N - 1)))
        return c

    def hard_rows(self, x, u):
        """formKKTSystemBlocks' hard rows (:238-248, 262-270) per knot as (column in [x_k; u_k], sign, value):
        the constraint hooks' jacobian rows must be box rows (one +-1 entry; a zero row is FULL_SET's
        inactive entry, sign 0).  Also sets the per-knot active-set bitmasks of the trace (bit t * 2n + e,
        include/tmpc.h) for rows over [q; qd; u]."""
        N, nx, n, nu = self.N, self.nx, self.n, self.nu
        con = self.s.other_constraints
        rows = [[] for _ in range(N)]
        self.mask = np.zeros(N, dtype=np.uint64)
        if not self.hard or con.total_hard_constraints(x, u) == 0:
            return rows
        for k in range(N):
            if not con.total_hard_constraints(x, u, k):
                continue
            if k < N - 1:
                jac = con.jacobian_hard_constraints(x[:, k], u[:, k], k)
                val = con.value_hard_constraints(x[:, k], u[:, k], k)
                width = n
            else:
                jac = con.jacobian_hard_constraints(x[:, N - 1], timestep=N - 1)
                val = con.value_hard_constraints(x[:, N - 1], timestep=N - 1)
                width = nx
            if val is None or not len(val):
                continue
            val = np.asarray(val, dtype=np.float64).reshape(-1)
            J = np.reshape(np.asarray(jac, dtype=np.float64), (len(val), width))
            for r in range(len(val)):
                nzc = np.nonzero(J[r])[0]
                if len(nzc) == 0:
                    rows[k].append((0, 0.0, float(val[r])))
                    continue
                if len(nzc) != 1 or abs(J[r, nzc[0]]) != 1.0:
                    raise NotImplementedError(
                        f"plugin-hook SQP: hard row {r} of knot {k} is not a box row (one +-1 entry of [x_k; u_k]); "
                        "the banded device QP takes the rows BoxConstraint forms")
                col, sg = int(nzc[0]), float(J[r, nzc[0]])
                rows[k].append((col, sg, float(val[r])))
                t, i = divmod(col, nu)
                self.mask[k] |= np.uint64(1) << np.uint64(t * 2 * nu + (i if sg > 0 else nu + i))
        return rows

    def blocks(self, x, u, xs):
        """formKKTSystemBlocks (:200-271) per knot: G [N][n][n], g [N][n], A, B, c."""
        N, nx, n = self.N, self.nx, self.n
        cost, con = self.s.cost, self.s.other_constraints
        f, A, Bm = self._step(x, u, True)
        G = np.zeros((N, n, n))
        g = np.zeros((N, n))
        c = np.zeros((N, nx))
        c[0] = x[:, 0] - xs
        kw = dict(iter_1=self.it, iter_2=self.outer, iter_3=self.ls)
        for k in range(N - 1):
            G[k] = cost.hessian(x[:, k], u[:, k], k, **kw)
            g[k] = np.asarray(cost.gradient(x[:, k], u[:, k], k, **kw)).reshape(-1)
            if con.total_soft_constraints(timestep=k) > 0:
                gck = np.asarray(con.jacobian_soft_constraints(x[:, k], u[:, k], k)).reshape(-1)
                g[k] = g[k] + gck
                G[k] += soft_hessian(con, x[:, k], u[:, k], k, gck)
            c[k + 1] = x[:, k + 1] - f[k]
        G[N - 1, :nx, :nx] = cost.hessian(x[:, N - 1], timestep=N - 1, **kw)
        g[N - 1, :nx] = np.asarray(cost.gradient(x[:, N - 1], timestep=N - 1, **kw)).reshape(-1)
        if con.total_soft_constraints(timestep=N - 1) > 0:
            gc = np.asarray(con.jacobian_soft_constraints(x[:, N - 1], timestep=N - 1)).reshape(-1)[:nx]
            g[N - 1, :nx] = g[N - 1, :nx] + gc
            G[N - 1, :nx, :nx] = G[N - 1, :nx, :nx] + soft_hessian(con, x[:, N - 1], None, N - 1, gc)[:nx, :nx]
        return G, g, A, Bm, c

    def directional(self, x_new, u_new, dxul):
        """D = sum_k grad(x_new, u_new) . dxul_k (+ soft jacobians) (:635-648)"""
        N, nx, n = self.N, self.nx, self.n
        cost, con = self.s.cost, self.s.other_constraints
        D = 0
        for k in range(N - 1):
            D += float(np.asarray(cost.gradient(x_new[:, k], u_new[:, k], k, self.it, self.outer, self.ls))
                       @ dxul[n * k:n * (k + 1), 0])
            if con.total_soft_constraints(timestep=k) > 0:
                D += float(np.asarray(con.jacobian_soft_constraints(x_new[:, k], u_new[:, k], k)).reshape(-1)
                           .dot(dxul[n * k:n * (k + 1), 0]))
        D += float(np.asarray(cost.gradient(x_new[:, N - 1], timestep=N - 1, iter_1=self.it, iter_2=self.outer,
                                            iter_3=self.ls)) @ dxul[n * (N - 1):n * (N - 1) + nx, 0])
        if con.total_soft_constraints(timestep=N - 1) > 0:
            D += float(np.asarray(con.jacobian_soft_constraints(x_new[:, N - 1], timestep=N - 1)).reshape(-1)[:nx]
                       .dot(dxul[n * (N - 1):n * (N - 1) + nx, 0]))
        return D

    def qp(self, x, u, xs, rho):
        G, g, A, Bm, c = self.blocks(x, u, xs)
        if self.banded:   # hard rows (the constraint hooks') and / or past 1024 Schur rows
            rows = self.hard_rows(x, u)
            r = self.ctx.qp_blocks_banded_batch(G[None], g[None], A[None], Bm[None], c[None], rho, [rows],
                                                self.method)
            self.singular = int(r["singular"][0])
        else:
            r = self.ctx.qp_blocks_batch(G[None], g[None], A[None], Bm[None], c[None], rho, self.method)
        return r["dxul"][0].reshape(-1, 1), int(r["pcg_iters"][0])

    # -- the loop
    def solve(self, x, u):
        o, N, nx, n = self.o, self.N, self.nx, self.n
        s = self.s
        x = np.array(x, dtype=np.float64)
        u = np.array(u, dtype=np.float64)
        xs = copy.deepcopy(x[:, 0])
        W = int(o["max_iter_SQP_DDP"]) + 1
        self.outer = 0
        exit_sqp = exit_soft = 0
        while True:
            rho, drho = o["rho_init_SQP_DDP"], 1
            J = self.total_cost(x, u)   # the previous pass's iteration / line-search indices (:541-542)
            c = self.violation(x, u, xs)
            self.it = 0                 # matrix_.iteration = 0 (:572)
            mu = 10   # :545-546
            merit = J + mu * c
            trace = [dict(iteration=0, line_search_iteration=0, alpha=1.0, rho=rho, J=J, c=c, merit=merit,
                          D=np.nan, reduction_ratio=np.nan, succeeded_line_search=0, pcg_iters=0, singular=0,
                          hard_active=np.zeros(N, dtype=np.uint64))]
            while True:
                dxul, inner = self.qp(x, u, xs, rho)   # formKKTSystemBlocks sees the last line search's index
                self.ls = 0                            # matrix_.line_search_iteration = 0 (:608)
                alpha, error = 1.0, False
                while True:
                    x_new, u_new = copy.deepcopy(x), copy.deepcopy(u)
                    for k in range(N):
                        x_new[:, k] = x_new[:, k] - alpha * dxul[n * k:n * k + nx, 0]
                        if k < N - 1:
                            u_new[:, k] = u_new[:, k] - alpha * dxul[n * k + nx:n * (k + 1), 0]
                    J_new = self.total_cost(x_new, u_new)
                    c_new = self.violation(x_new, u_new, xs)
                    D = self.directional(x_new, u_new, dxul)
                    merit_new = J_new + mu * c_new
                    delta_J = J - J_new
                    delta_merit = merit - merit_new
                    with np.errstate(divide="ignore", invalid="ignore"):
                        ratio = np.float64(delta_merit) / np.float64(alpha * (D - mu * c_new))
                    if (delta_merit >= 0 and ratio >= o["expected_reduction_min_SQP_DDP"]
                            and ratio <= o["expected_reduction_max_SQP_DDP"]):
                        x, u, J, c, merit = x_new, u_new, J_new, c_new, merit_new
                        rho, drho = s.reduce_regularization(rho, drho, o)
                        trace.append(dict(iteration=self.it, line_search_iteration=self.ls, alpha=alpha, rho=rho,
                                          J=J, c=c, merit=merit, D=D, reduction_ratio=ratio,
                                          succeeded_line_search=1, pcg_iters=inner, singular=self.singular,
                                          hard_active=self.mask.copy()))
                        break
                    elif alpha > o["alpha_min_SQP_DDP"]:
                        alpha *= o["alpha_factor_SQP_DDP"]
                        self.ls += 1
                    else:
                        error = True
                        trace.append(dict(iteration=self.it, line_search_iteration=self.ls, alpha=alpha, rho=rho,
                                          J=J, c=c, merit=merit, D=D, reduction_ratio=ratio,
                                          succeeded_line_search=0, pcg_iters=inner, singular=self.singular,
                                          hard_active=self.mask.copy()))
                        break
                exit_flag, self.it, rho, drho = s.check_for_exit_or_error(error, delta_J, self.it, rho, drho, o)
                if exit_flag:
                    exit_sqp = s.exit_sqp
                    break
            exit_flag, self.outer = s.check_and_update_soft_constraints(x, u, self.outer, o)
            if exit_flag:
                exit_soft = s.exit_soft
                break
        tr = {k: np.zeros(W, dtype=np.int32 if k in ("iteration", "line_search_iteration", "succeeded_line_search",
                                                       "pcg_iters", "singular") else np.float64)
              for k in trace[0] if k != "hard_active"}
        tr["hard_active"] = np.zeros((W, N), dtype=np.uint64)
        for i, row in enumerate(trace[:W]):
            for k, v in row.items():
                tr[k][i] = v
        return dict(x=x, u=u, exit_sqp=exit_sqp, exit_soft=exit_soft, outer_iter=self.outer, sqp_iter=self.it,
                    trace=tr)


def sqp_hooks_batch(solver, ctx, x, u, N, dt, method, options):
    """SQP_batch over plugin hooks: the problems one after another (their hooks are the caller's Python),
    each QP on the GPU.  Returns SQP_batch's dict."""
    p = solver.plant
    nx, nu = p.get_num_pos() + p.get_num_vel(), p.get_num_cntrl()
    if nx != 2 * nu or not 1 <= nu <= 7:
        raise NotImplementedError(f"plugin-hook SQP: the device QP takes nx = 2 nu with 1 <= nu <= 7 "
                                  f"(got nx = {nx}, nu = {nu})")
    if options.get("precision", "fp64") != "fp64":
        raise NotImplementedError("the fp32 / mixed precision modes need device plugins")
    if options.get("pcg_warm_start"):
        raise NotImplementedError("pcg_warm_start needs device plugins")
    con = solver.other_constraints
    if any(c.is_hard_constraint_mode() for _, c in con.limits()) and method.startswith("PCG") and \
            any(c.mode == "FULL_SET" for _, c in con.limits() if c.is_hard_constraint_mode()):
        raise NotImplementedError("FULL_SET box constraints with a PCG method: the inactive rows of C are zero, so S "
                                  "is singular and the reference's preconditioner raises LinAlgError; use method S")
    B = x.shape[0]
    outs = [_HookSQP(solver, ctx, N, dt, method, options).solve(x[b], u[b]) for b in range(B)]
    r = {k: np.array([o[k] for o in outs], dtype=np.int32) for k in ("exit_sqp", "exit_soft", "outer_iter",
                                                                       "sqp_iter")}
    r["x"] = np.array([o["x"] for o in outs])
    r["u"] = np.array([o["u"] for o in outs])
    r["trace"] = {k: np.array([o["trace"][k] for o in outs]) for k in outs[0]["trace"]}
    return r
