"""CPU, world_size 2: the multi-GPU path of bench.py (trajoptmpcreference_amd/dist.py) --
rank 0 draws every rank's start states and broadcasts them, each rank solves its
contiguous slice, the per-problem summaries are gathered in rank order and the
timed region is the max over ranks.

On the GPUs the collectives are RCCL through libtmpc (dist.make_comm ->
_native.Comm); here the same dist functions run over a gloo-backed stand-in
with the same four methods, and the per-rank "solver" is the oracle (real SQP
solves, oracle-sized) -- so the test checks the sharding logic end to end:
sharded results equal the single-process results bitwise."""
import multiprocessing as mp
import os
import socket

import numpy as np

import bench
from trajoptmpcreference_amd import dist


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class GlooComm:
    """Test-side stand-in for _native.Comm (broadcast / allgather / max / barrier) over gloo."""

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


def _solve_slice(q0, n, N, dt):
    """The per-rank solve: oracle SQP-PCG-SS on each problem of the slice."""
    from oracle import sqp as osqp
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    m = parse_urdf(planar_arm_urdf(n))
    cost = osqp.QuadCost(np.eye(2 * n), 100 * np.eye(2 * n), 0.1 * np.eye(n), np.zeros(2 * n))
    ex, it, xs = [], [], []
    for q in q0:
        x = np.zeros((2 * n, N))
        x[:n, 0] = q
        u = np.zeros((n, N - 1))
        from oracle import rbd
        for k in range(N - 1):
            x[:, k + 1] = rbd.euler(m, x[:, k][None], u[:, k][None], dt)[0]
        r = osqp.sqp(m, cost, x, u, N, dt, "PCG-SS")
        ex.append(r["exit_sqp"])
        it.append(r["sqp_iter"])
        xs.append(r["x"])
    return np.array(ex, dtype=np.int32), np.array(it, dtype=np.int32), np.array(xs)


def _worker(rank, world, port, B, n, N, seed0, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    try:
        comm = GlooComm(world, rank)
        assert dist.env_ranks() == (rank, world, rank)
        q0 = dist.scatter_from_root(comm, rank, B, lambda count: bench.initial_states(n, count, seed0), (n,))
        comm.barrier()
        ex, it, xs = _solve_slice(q0, n, N, 0.1)
        g = dist.gather_summaries(comm, exit_codes=ex, iters=it, x=xs)
        elapsed = comm.max(0.25 + rank)   # rank-dependent "time"
        comm.barrier()
        comm.close()
        q.put((rank, q0, g, elapsed))
    except Exception as e:  # surface the failure in the parent
        import traceback
        q.put((rank, traceback.format_exc(), None, None))


def test_two_rank_sharded_solves_equal_single_process():
    world, B, n, N, seed0 = 2, 2, 2, 8, 11
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, n, N, seed0, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    q_all = bench.initial_states(n, world * B, seed0)
    ex_ref, it_ref, x_ref = _solve_slice(q_all, n, N, 0.1)
    for rank, q0, g, elapsed in out:
        assert not isinstance(q0, str), q0
        lo, hi = dist.shard_range(rank, B)
        # the broadcast start states are the single-process workload's slice for this rank
        assert np.array_equal(q0, q_all[lo:hi])
        # gathered results, in rank order, equal the single-process solves bitwise
        assert np.array_equal(g["exit_codes"], ex_ref)
        assert np.array_equal(g["iters"], it_ref)
        assert np.array_equal(g["x"], x_ref)
        # every rank sees the slowest rank's time
        assert elapsed == 1.25


def test_single_rank_comm_is_a_no_op():
    c = dist.LocalComm()
    c.barrier()
    assert c.max(3.5) == 3.5
    a = np.arange(6.0).reshape(3, 2)
    assert np.array_equal(c.broadcast(a), a)
    assert c.allgather(a).shape == (1, 3, 2)
    g = dist.gather_summaries(c, e=np.array([1, 2], dtype=np.int32))
    assert np.array_equal(g["e"], [1, 2])
    q0 = dist.scatter_from_root(c, 0, 4, lambda count: bench.initial_states(3, count, 5), (3,))
    assert np.array_equal(q0, bench.initial_states(3, 4, 5))
    assert dist.shard_range(3, 100) == (300, 400)
    c.close()


def test_unique_id_file_exchange(tmp_path, monkeypatch):
    """TMPC_COMM_ID_FILE set by the launcher: rank 0 publishes the RCCL id atomically; another rank reads
    exactly those bytes (the id itself comes from libtmpc on the GPU box: faked here)."""
    path = tmp_path / "uid"
    monkeypatch.setenv("TMPC_COMM_ID_FILE", str(path))
    fake = bytes(range(128))
    assert dist.exchange_unique_id(0, 2, make_id=lambda: fake) == fake
    assert dist.exchange_unique_id(1, 2, timeout_s=5, make_id=lambda: fake) == fake


_RANK_SCRIPT = """
import os, sys
sys.path.insert(0, {root!r})
from trajoptmpcreference_amd import dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
cfg = dist.config_hash({{"B": 4096, "N": int(os.environ["TEST_N"])}})
try:
    uid = dist.exchange_unique_id(rank, world, cfg, timeout_s=60, make_id=lambda: bytes(range(7, 135)))
    print("OK", os.getppid(), uid.hex())
except RuntimeError as e:
    print("REFUSED", os.getppid(), e)
"""


def _launch_ranks(world, port, Ns):
    """world processes with DIFFERENT parents: rank 0 a child of this test process, the others children of
    their own `bash -c` (so nothing keyed on the parent pid could pair them)."""
    import subprocess
    import sys
    from conftest import ROOT
    script = _RANK_SCRIPT.format(root=ROOT)
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world),
                   TEST_N=str(Ns[r]))
        env.pop("TMPC_COMM_ID_FILE", None)
        cmd = [sys.executable, "-c", script]
        if r:
            cmd = ["bash", "-c", 'exec_py="$0"; "$exec_py" -c "$1"; true', sys.executable, script]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    return [p.communicate(timeout=120)[0].strip().splitlines()[-1] for p in procs]


def test_unique_id_tcp_exchange_across_process_trees():
    """The RCCL id over TCP at MASTER_ADDR : MASTER_PORT + 1 (dist.exchange_unique_id): every rank gets
    rank 0's id, whatever the process tree (the ranks here have different parents)."""
    port = _free_port()
    out = _launch_ranks(3, port - 1, [64, 64, 64])
    assert all(line.startswith("OK") for line in out), out
    assert len({line.split()[2] for line in out}) == 1
    assert len({line.split()[1] for line in out}) == 3      # three different parent pids


def test_mismatched_configuration_fails_fast():
    """A rank whose configuration hash differs from rank 0's is refused, and rank 0 raises too."""
    port = _free_port()
    out = _launch_ranks(2, port - 1, [64, 32])
    assert out[0].startswith("REFUSED") and "ranks [1]" in out[0], out
    assert out[1].startswith("REFUSED"), out


def test_one_mismatched_rank_refuses_every_rank():
    """World 3, rank 2 mismatched: the matching rank 1 must be refused too (rank 0 answers only after it
    has read every request), so no rank goes on to the RCCL communicator init and blocks there."""
    port = _free_port()
    out = _launch_ranks(3, port - 1, [64, 64, 32])
    assert all(line.startswith("REFUSED") for line in out), out
    assert "ranks [2]" in out[0], out


def _run_bench(args, extra_env=None, timeout=300):
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT", "TMPC_COMM_ID_FILE")}
    env.update(TMPC_BENCH_STANDIN=os.path.join(ROOT, "tests", "bench_standin.py"), OMP_NUM_THREADS="1")
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2` with no launcher starts the two ranks itself (the driver's command form):
    one line from rank 0 with n_gpus 2, the global batch, and every problem's exit code / iteration count
    gathered from both ranks -- equal to the single-process solves of the same workload (stand-in GPU
    context and gloo collectives: tests/bench_standin.py)."""
    from oracle import sqp as osqp
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    B, n, N = 2, 2, 8
    args = ["--gpus", "2", "--batch", str(B), "--links", str(n), "--N", str(N), "--steps", "1", "--warmup", "0"]
    rc, line, err = _run_bench(args)
    assert rc == 0, err[-3000:]
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 2 * B and line["problems_gathered"] == 2 * B
    assert line["scaling"] == "weak" and line["value"] > 0
    m = parse_urdf(planar_arm_urdf(n))
    cost = osqp.QuadCost(np.eye(2 * n), 100 * np.eye(2 * n), 0.1 * np.eye(n), np.zeros(2 * n))
    q0 = bench.initial_states(n, 2 * B, 0)
    codes, iters = {}, []
    for q in q0:
        x = np.zeros((2 * n, N))
        x[:n, 0] = q
        from oracle import rbd
        for k in range(N - 1):
            x[:, k + 1] = rbd.euler(m, x[:, k][None], np.zeros((1, n)), 0.1)[0]
        r = osqp.sqp(m, cost, x, np.zeros((n, N - 1)), N, 0.1, "PCG-SS")
        codes[str(r["exit_sqp"])] = codes.get(str(r["exit_sqp"]), 0) + 1
        iters.append(r["sqp_iter"])
    assert line["exit_codes"] == codes
    assert line["iters_mean"] == float(np.mean(iters)) and line["iters_max"] == max(iters)


def test_bench_fails_when_a_rank_fails():
    rc, line, err = _run_bench(["--gpus", "2", "--batch", "2", "--links", "2", "--N", "8", "--steps", "1",
                                "--warmup", "0"], extra_env={"TMPC_STANDIN_FAIL_RANK": "1"}, timeout=200)
    assert rc != 0 and "ranks [0, 1] failed" in err and "fails on purpose" in err, (rc, err[-2000:])


def test_bench_world_size_must_match_gpus():
    rc, line, err = _run_bench(["--gpus", "2", "--batch", "2", "--links", "2", "--N", "8"],
                               extra_env={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert rc != 0 and "WORLD_SIZE=3 but --gpus 2" in err, err[-2000:]
