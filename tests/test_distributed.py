"""CPU, world_size 2 over gloo: the multi-GPU path of bench.py (one process per
GPU, contiguous disjoint problem slices, barrier + max over ranks of the timed
region, no data-path collective) run with the gloo backend."""
import multiprocessing as mp
import os
import socket

import numpy as np

import bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, n, seed0, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        comm = bench.Comm(world, rank, backend="gloo")
        comm.barrier()
        q0 = bench.initial_states(n, B, bench.shard_seed_base(seed0, rank, B))
        import torch
        parts = [torch.zeros(B, n, dtype=torch.float64) for _ in range(world)]
        comm.tdist.all_gather(parts, torch.from_numpy(q0))   # test-side check only
        elapsed = comm.max(0.25 + rank)                       # rank-dependent "time"
        comm.barrier()
        comm.close()
        q.put((rank, np.concatenate([p.numpy() for p in parts]), elapsed))
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e), None))


def test_two_rank_sharding_and_max_time():
    world, B, n, seed0 = 2, 5, 6, 11
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, n, seed0, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    ref = bench.initial_states(n, world * B, seed0)
    for rank, gathered, elapsed in out:
        assert not isinstance(gathered, str), gathered
        # the ranks' slices tile the single-process workload exactly, in rank order
        assert np.array_equal(gathered, ref)
        # every rank sees the slowest rank's time
        assert elapsed == 1.25


def test_single_rank_comm_is_a_no_op():
    c = bench.Comm(1, 0)
    c.barrier()
    assert c.max(3.5) == 3.5
    c.close()
    assert bench.shard_seed_base(7, 3, 100) == 307
