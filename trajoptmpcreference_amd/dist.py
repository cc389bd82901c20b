"""Sharding independent problem batches across the GPUs of one node.

The reference has no distributed path: its drivers solve independent problems
in a multiprocessing.Pool (examples/test_multiple.py:123-128).  Here one process
per GPU (any launcher that starts N processes and sets RANK / WORLD_SIZE /
LOCAL_RANK, e.g. ``python -m torch.distributed.run``) solves a contiguous,
disjoint slice of one global batch -- weak scaling, no exchange inside a solve.
RCCL over xGMI (``_native.Comm``, the tmpc_comm_* C ABI; no PyTorch) carries
the initial states broadcast from rank 0 and the per-problem result summaries
gathered back; the max over ranks of the timed region uses the same
communicator.

The RCCL unique id is handed from rank 0 to the other ranks through a file
next to the launcher: its name includes MASTER_PORT and the parent (launcher)
pid that the ranks of one launch share.
"""
import os
import time

import numpy as np

from . import _native


def env_ranks():
    """(rank, world, local_rank) from the launcher's environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(rank: int, B: int):
    """Rank r owns global problems [r B, (r + 1) B): contiguous, disjoint, in rank order, so every
    rank's results equal the single-process results for the same problems."""
    return rank * B, (rank + 1) * B


def _id_path():
    p = os.environ.get("TMPC_COMM_ID_FILE")
    if p:
        return p
    return f"/tmp/tmpc_rccl_id_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}"


def exchange_unique_id(rank: int, timeout_s: float = 120.0) -> bytes:
    """Rank 0 creates the RCCL unique id and publishes it atomically; the others wait for it."""
    path = _id_path()
    if rank == 0:
        uid = _native.comm_unique_id()
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    t0 = time.time()
    while True:
        try:
            with open(path, "rb") as f:
                uid = f.read()
            if len(uid) == _native.COMM_ID_BYTES:
                return uid
        except FileNotFoundError:
            pass
        if time.time() - t0 > timeout_s:
            raise TimeoutError(f"rank {rank}: no RCCL unique id at {path} after {timeout_s} s")
        time.sleep(0.05)


class LocalComm:
    """World size 1: the collectives are identities (no RCCL communicator needed)."""
    world, rank = 1, 0

    def barrier(self):
        pass

    def broadcast(self, arr, root=0):
        return np.array(arr, copy=True)

    def allgather(self, arr):
        return np.asarray(arr)[None].copy()

    def max(self, v):
        return float(v)

    def close(self):
        pass


def make_comm(ctx, rank: int, world: int):
    """RCCL communicator for world > 1 (one rank per GPU), LocalComm otherwise."""
    if world == 1:
        return LocalComm()
    uid = exchange_unique_id(rank)
    comm = _native.Comm(ctx, world, rank, uid)
    comm.barrier()
    if rank == 0:
        try:
            os.remove(_id_path())
        except OSError:
            pass
    return comm


def scatter_from_root(comm, rank: int, B: int, make_global, tail_shape, dtype=np.float64):
    """Rank 0 builds the global [world B, *tail_shape] array (make_global(count)), every rank
    receives it by broadcast and keeps its own slice ('ncclBroadcast ... of all
    initial states').  The other ranks never call make_global."""
    shape = (comm.world * B,) + tuple(tail_shape)
    glob = np.ascontiguousarray(make_global(shape[0]), dtype=dtype) if rank == 0 else np.empty(shape, dtype)
    if glob.shape != shape:
        raise ValueError(f"make_global returned {glob.shape}, expected {shape}")
    glob = comm.broadcast(glob, root=0)
    lo, hi = shard_range(rank, B)
    return glob[lo:hi].copy()


def gather_summaries(comm, **arrays):
    """Per-problem [B] arrays of every rank -> global [world B] arrays (rank order) on every rank."""
    out = {}
    for k, v in arrays.items():
        g = comm.allgather(np.ascontiguousarray(v))
        out[k] = g.reshape((-1,) + g.shape[2:])
    return out
