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

The RCCL unique id travels from rank 0 to the other ranks over a TCP socket at
MASTER_ADDR : MASTER_PORT + 1 (TMPC_COMM_PORT overrides the port), so any
launcher that exports the usual rendezvous variables works, whatever the
process tree.  Every rank sends a hash of its run configuration (batch size,
horizon, model, cost, options, limits) with its request; rank 0 refuses a
mismatch and every rank fails fast instead of solving different problems.
A launcher that prefers a shared file sets TMPC_COMM_ID_FILE.
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


def config_hash(*parts) -> bytes:
    """sha256 over the run configuration: numpy arrays (shape, dtype, bytes), bytes, or anything JSON-able."""
    import hashlib
    import json
    h = hashlib.sha256()
    for p in parts:
        if isinstance(p, np.ndarray):
            h.update(repr((p.shape, p.dtype.str)).encode())
            h.update(np.ascontiguousarray(p).tobytes())
        elif isinstance(p, (bytes, bytearray)):
            h.update(bytes(p))
        else:
            h.update(json.dumps(p, sort_keys=True, default=str).encode())
    return h.digest()


def _comm_addr():
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("TMPC_COMM_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
    return host, port


def _recv_exact(sock, n):
    buf = b""
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("peer closed the RCCL id exchange")
        buf += chunk
    return buf


def exchange_unique_id(rank: int, world: int, cfg: bytes = b"\0" * 32, timeout_s: float = 120.0,
                       make_id=None) -> bytes:
    """Rank 0 creates the RCCL unique id (make_id, default ncclGetUniqueId) and serves it over TCP to
    the world - 1 other ranks, each of which first sends (rank, cfg).  Rank 0 reads every request before
    it answers any: if every cfg equals its own, every rank gets the id; if any differs, every rank gets
    a refusal and raises (rank 0 too), so no rank is left waiting in the communicator init.  With TMPC_COMM_ID_FILE
    set, the id goes through that file instead (no config check)."""
    import socket
    import struct
    make_id = make_id or _native.comm_unique_id
    if len(cfg) != 32:
        raise ValueError("cfg must be a 32-byte digest (config_hash)")
    path = os.environ.get("TMPC_COMM_ID_FILE")
    if path:
        return _exchange_via_file(rank, path, timeout_s, make_id)
    host, port = _comm_addr()
    n_id = _native.COMM_ID_BYTES
    if rank == 0:
        uid = make_id()
        bad = []
        conns = []
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as srv:
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((host, port))
            srv.listen(max(1, world))
            srv.settimeout(timeout_s)
            try:
                # every request first (connections held open), then one verdict for all: the id to every
                # rank, or a refusal to every rank -- no rank may go on to the communicator init alone
                for _ in range(world - 1):
                    conn, _ = srv.accept()
                    conns.append(conn)
                    conn.settimeout(timeout_s)
                    r, peer_cfg = struct.unpack("<i32s", _recv_exact(conn, 36))
                    if peer_cfg != cfg:
                        bad.append(r)
                reply = (b"\x01" + cfg + b"\0" * (n_id - 32)) if bad else (b"\x00" + uid)
                for conn in conns:
                    conn.sendall(reply)
            finally:
                for conn in conns:
                    conn.close()
        if bad:
            raise RuntimeError(f"rank 0: ranks {sorted(bad)} run a different configuration "
                               "(batch / horizon / model / cost / options / limits); refusing to start")
        return uid
    t0 = time.time()
    while True:
        try:
            with socket.create_connection((host, port), timeout=5.0) as c:
                c.settimeout(timeout_s)
                c.sendall(struct.pack("<i32s", rank, cfg))
                reply = _recv_exact(c, 1 + n_id)
            break
        except (ConnectionRefusedError, socket.timeout, OSError):
            if time.time() - t0 > timeout_s:
                raise TimeoutError(f"rank {rank}: no RCCL id server at {host}:{port} after {timeout_s} s")
            time.sleep(0.05)
    if reply[0] != 0:
        raise RuntimeError(f"rank {rank}: rank 0 runs a different configuration "
                           "(batch / horizon / model / cost / options / limits); refusing to start")
    return reply[1:]


def _exchange_via_file(rank, path, timeout_s, make_id):
    if rank == 0:
        uid = make_id()
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


def make_comm(ctx, rank: int, world: int, cfg: bytes = b"\0" * 32):
    """RCCL communicator for world > 1 (one rank per GPU), LocalComm otherwise.  cfg: config_hash of
    the run; every rank must pass the same one."""
    if world == 1:
        return LocalComm()
    uid = exchange_unique_id(rank, world, cfg)
    comm = _native.Comm(ctx, world, rank, uid)
    comm.barrier()
    path = os.environ.get("TMPC_COMM_ID_FILE")
    if rank == 0 and path:
        try:
            os.remove(path)
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
