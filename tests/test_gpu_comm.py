"""GPU: the RCCL communicator behind tmpc_comm_* (the multi-GPU path of bench.py).

The box has one GPU and RCCL refuses two ranks on one device, so the
collectives run as a 1-rank communicator here (the world-size-2 logic is
covered on CPU by test_distributed.py; the driver's 8-GPU run exercises the
rest)."""
import numpy as np
import pytest

from trajoptmpcreference_amd import _native, dist

pytestmark = pytest.mark.gpu


def test_rccl_one_rank_collectives(ctx):
    uid = _native.comm_unique_id()
    assert len(uid) == _native.COMM_ID_BYTES
    comm = _native.Comm(ctx, 1, 0, uid)
    try:
        comm.barrier()
        a = np.arange(12, dtype=np.float64).reshape(3, 4)
        assert np.array_equal(comm.broadcast(a, root=0), a)
        g = comm.allgather(np.array([3, 1, 4], dtype=np.int32))
        assert g.shape == (1, 3) and list(g[0]) == [3, 1, 4]
        assert comm.max(2.5) == 2.5
        q0 = dist.scatter_from_root(comm, 0, 5, lambda count: np.arange(count * 2, dtype=np.float64).reshape(count, 2),
                                    (2,))
        assert np.array_equal(q0, np.arange(10.0).reshape(5, 2))
        s = dist.gather_summaries(comm, e=np.array([2, 2, 1], dtype=np.int32))
        assert list(s["e"]) == [2, 2, 1]
    finally:
        comm.close()
