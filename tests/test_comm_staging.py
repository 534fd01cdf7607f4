"""Host-staged point-to-point / all-to-all (gloo ranks that keep buffers on a GPU; here the
staging path is forced on CPU tensors): rotation and sparse push/pull give the same results."""
import torch

from harp_amd.runtime.launcher import launch


def _worker(comm):
    from harp_amd.runtime.dymoro import DeviceRotator

    out = {}
    for stage in (False, True):
        comm.stage = stage
        P, r = comm.world_size, comm.rank
        slabs = [torch.full((4, 3), float(10 * r + k)) for k in range(2)]
        rot = DeviceRotator(comm, slabs, name=f"st{int(stage)}")
        for k in range(2):
            rot.start(k, [(q + 1) % P for q in range(P)])
        got = [float(rot.get(k)[0, 0]) for k in range(2)]
        recv = torch.empty(P * 2, dtype=torch.int64)
        comm.all_to_all_single(recv, torch.arange(P * 2, dtype=torch.int64) + 100 * r)
        out[stage] = (got, recv.tolist())
    comm.stage = False
    return out


def test_staged_p2p_matches_direct():
    for o in launch(_worker, 3, timeout=300):
        assert o[False] == o[True]
