"""Python session API (numpy collectives, homogeneous / heterogeneous partitioning) and
HarpDAALComm object communication on 3 gloo workers."""
import numpy as np
import torch

from harp_amd.parallel.daal_comm import HarpDAALComm
from harp_amd.runtime.launcher import launch
from harp_amd.session import HarpSession, PartitioningMode, Type


def _session_job(comm):
    s = HarpSession("t", comm=comm)
    me, P = s.self_id, s.num_workers
    out = {}
    out["bcast"] = s.com.broadcast("c", "b", np.arange(6.0).reshape(2, 3) if me == 1 else None, Type.DOUBLE,
                                   PartitioningMode.HOMOGENEOUS, 1)
    out["bcast_het"] = s.com.broadcast("c", "bh", {7: np.ones(3), 9: np.arange(5)} if me == 0 else None, Type.INT,
                                       PartitioningMode.HETEROGENEOUS, 0)
    out["allreduce"] = s.com.allreduce("c", "a", np.full((2, 4), me + 1.0), Type.FLOAT)
    out["reduce"] = s.com.reduce("c", "r", np.full(3, me + 1), Type.LONG, root=2)
    out["allgather"] = s.com.allgather("c", "g", {me: np.full(2, me)}, Type.INT)
    out["regroup"] = s.com.regroup("c", "rg", {k: np.ones(2) for k in range(6)})
    out["rotate"] = s.com.rotate("c", "rt", {me: np.full(1, me)}, Type.INT)
    assert s.com.barrier()
    d = HarpDAALComm(comm)
    out["daal_b"] = d.harpdaal_braodcast(torch.arange(3) if me == 0 else None)
    out["daal_g"] = d.harpdaal_gather(torch.tensor([me]))
    out["daal_ag"] = d.harpdaal_allgather(torch.tensor([me * 10]))
    return out


def test_session_and_daal_comm():
    res = launch(_session_job, 3, timeout=300)
    for r, o in enumerate(res):
        assert np.array_equal(o["bcast"], np.arange(6.0).reshape(2, 3))
        assert sorted(o["bcast_het"]) == [7, 9] and o["bcast_het"][9].dtype == np.int32
        assert np.allclose(o["allreduce"], 6.0) and o["allreduce"].dtype == np.float32
        assert (o["reduce"] is None) == (r != 2)
        assert sorted(o["allgather"]) == [0, 1, 2]
        assert all(k % 3 == r for k in o["regroup"]) and all(np.allclose(v, 3) for v in o["regroup"].values())
        assert list(o["rotate"]) == [(r - 1) % 3]
        assert torch.equal(o["daal_b"], torch.arange(3))
        assert [int(x) for x in o["daal_ag"]] == [0, 10, 20]
    assert res[2]["reduce"].tolist() == [6, 6, 6]
    assert [int(x) for x in res[0]["daal_g"]] == [0, 1, 2] and res[1]["daal_g"] is None


def test_single_worker_session():
    s = HarpSession("solo")
    assert s.num_workers == 1 and s.name == "solo"
    assert np.array_equal(s.com.allreduce("c", "a", np.ones((2, 2))), np.ones((2, 2)))
