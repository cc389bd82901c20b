"""Test stand-in for bench.py's GPU context and RCCL communicator (TMPC_BENCH_STANDIN, bench._standin):
lets the CPU suite run `bench.py --gpus 2` end to end -- the rank launcher, the RCCL-id / config-hash
exchange, the broadcast of the start states, the per-rank solves, the gather and the JSON line --
without a GPU.  "Device memory" is host byte buffers; the solves are the oracle's (test infrastructure,
never loaded by the driver's runs); the collectives go over gloo with the same four methods as
_native.Comm."""
import os

import numpy as np

from trajoptmpcreference_amd import dist


class Context:
    options = b"bench-standin"

    def __init__(self, device=0):
        if os.environ.get("TMPC_STANDIN_FAIL_RANK") == os.environ.get("RANK"):
            raise RuntimeError(f"stand-in: rank {os.environ.get('RANK')} fails on purpose")
        self.device = device
        self.mem, self.next = {}, 1
        self.model = None
        self.counters = [0, 0, 0, 9]

    # configuration
    def set_model(self, model, gravity=-9.81):
        self.model = model

    def set_cost_quadratic(self, Q, QF, R, xg, QF_start=None):
        self.cost = (np.array(Q), np.array(QF), np.array(R), np.array(xg))

    def set_box_limits(self, spec):
        if spec:
            raise NotImplementedError("stand-in: no box limits")

    def set_options(self, **kw):
        pass

    def set_soft_state(self, *a):
        pass

    # memory
    def alloc(self, nbytes):
        h = self.next
        self.next += 1
        self.mem[h] = np.zeros(int(nbytes), dtype=np.uint8)
        return h

    def free(self, h):
        self.mem.pop(h, None)

    def h2d(self, dst, arr):
        b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        self.mem[dst][:b.size] = b

    def d2h(self, arr, src, offset=0):
        b = arr.view(np.uint8).reshape(-1)
        b[:] = self.mem[src][offset:offset + b.size]

    def d2d(self, dst, src, nbytes):
        self.mem[dst][:nbytes] = self.mem[src][:nbytes]

    def synchronize(self):
        pass

    def _view(self, h, shape):
        return self.mem[h][:8 * int(np.prod(shape))].view(np.float64).reshape(shape)

    # solves (the oracle)
    def rollout_device(self, B, N, dt, d_x, d_u):
        from oracle import rbd
        n = self.model.n
        x, u = self._view(d_x, (B, 2 * n, N)), self._view(d_u, (B, n, N - 1))
        for b in range(B):
            for k in range(N - 1):
                x[b, :, k + 1] = rbd.euler(self.model, x[b, :, k][None], u[b, :, k][None], dt)[0]

    def _solve(self, x, u, N, dt, method):
        from oracle import sqp as osqp
        Q, QF, R, xg = self.cost
        r = osqp.sqp(self.model, osqp.QuadCost(Q, QF, R, xg), x, u, N, dt, method)
        self.counters[0] += len(r["pcg_iters"])
        self.counters[1] += int(sum(r["pcg_iters"]))
        return r

    def sqp_solve_batch_device(self, B, N, dt, d_x, d_u, method="PCG-SS", want_status=False):
        n = self.model.n
        x, u = self._view(d_x, (B, 2 * n, N)), self._view(d_u, (B, n, N - 1))
        ex, it = np.zeros(B, dtype=np.int32), np.zeros(B, dtype=np.int32)
        for b in range(B):
            r = self._solve(x[b].copy(), u[b].copy(), N, dt, method)
            x[b], u[b] = r["x"], r["u"]
            ex[b], it[b] = r["exit_sqp"], r["sqp_iter"]
        return (ex, it) if want_status else (None, None)

    def solve_stream_device(self, solver, P, slots, N, dt, d_x_in, d_u_in, period, d_x_out=None, d_u_out=None,
                            d_status=None, d_trace=None, substreams=1):
        """the continuous-batching entry point's contract: problem p from input p % period, its results to
        output row p (the stand-in solves them one by one)"""
        n = self.model.n
        xi, ui = self._view(d_x_in, (period, 2 * n, N)), self._view(d_u_in, (period, n, N - 1))
        xo = self._view(d_x_out, (P, 2 * n, N)) if d_x_out else None
        uo = self._view(d_u_out, (P, n, N - 1)) if d_u_out else None
        st = self.mem[d_status][:16 * P].view(np.int32).reshape(P, 4) if d_status else None
        counters = [0, 0, 0, 9]
        for p in range(P):
            r = self._solve(xi[p % period].copy(), ui[p % period].copy(), N, dt, solver)
            counters[0] += len(r["pcg_iters"])
            counters[1] += int(sum(r["pcg_iters"]))
            if xo is not None:
                xo[p], uo[p] = r["x"], r["u"]
            if st is not None:
                st[p] = (r["exit_sqp"], r["sqp_iter"], r["exit_soft"], r["outer_iter"])
        self.counters = counters

    def sqp_solve_batch(self, x, u, N, dt, method="PCG-SS", with_trace=True, hard_active=False):
        rs = [self._solve(np.array(x[b]), np.array(u[b]), N, dt, method) for b in range(x.shape[0])]
        return dict(exit_sqp=np.array([r["exit_sqp"] for r in rs], dtype=np.int32),
                    sqp_iter=np.array([r["sqp_iter"] for r in rs], dtype=np.int32),
                    x=np.array([r["x"] for r in rs]), u=np.array([r["u"] for r in rs]), trace={})

    # statistics
    def reset_stats(self):
        self.counters = [0, 0, 0, 9]

    def solve_counters(self):
        c, self.counters = self.counters, [0, 0, 0, 9]
        return c

    def kernel_stats(self, name):
        return (1, 1.0) if name in ("qp", "ls_decide") else (0, 0.0)


class GlooComm:
    """_native.Comm's four collectives over torch.distributed gloo."""

    def __init__(self, world, rank):
        import torch
        import torch.distributed as tdist
        tdist.init_process_group(backend="gloo", world_size=world, rank=rank)
        self.torch, self.tdist, self.world, self.rank = torch, tdist, world, rank

    def barrier(self):
        self.tdist.barrier()

    def broadcast(self, arr, root=0):
        t = self.torch.from_numpy(np.ascontiguousarray(arr).copy())
        self.tdist.broadcast(t, src=root)
        return t.numpy()

    def allgather(self, arr):
        t = self.torch.from_numpy(np.ascontiguousarray(arr))
        parts = [self.torch.empty_like(t) for _ in range(self.world)]
        self.tdist.all_gather(parts, t)
        return np.stack([p.numpy() for p in parts])

    def max(self, v):
        t = self.torch.tensor([float(v)], dtype=self.torch.float64)
        self.tdist.all_reduce(t, op=self.tdist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        self.tdist.destroy_process_group()


def make_comm(ctx, rank, world, cfg):
    """The product's id / config-hash exchange (dist.exchange_unique_id, a fake id), then gloo."""
    if world == 1:
        return dist.LocalComm()
    dist.exchange_unique_id(rank, world, cfg, timeout_s=60, make_id=lambda: bytes(range(128)))
    return GlooComm(world, rank)
