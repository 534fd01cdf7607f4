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


def _dev_stage_worker(comm):
    """The nccl host-tensor path (device copies) forced on gloo CPU ranks, where the
    'device' is the host: every primitive must give the direct path's results."""
    out = {}
    P, r = comm.world_size, comm.rank
    for ds in (False, True):
        comm.dev_stage = ds
        res = []
        t = torch.arange(6, dtype=torch.float64) + r
        comm.all_reduce(t)
        res.append(t.tolist())
        b = torch.full((3,), float(r))
        comm.broadcast(b, 1)
        res.append(b.tolist())
        rd = torch.full((2,), float(r + 1))
        comm.reduce(rd, 0)
        res.append(rd.tolist() if r == 0 else None)
        ag = torch.empty(P * 2, dtype=torch.int64)
        comm.all_gather_into(ag, torch.tensor([r, 10 * r]))
        res.append(ag.tolist())
        a2a = torch.empty(P * 2, dtype=torch.int64)
        comm.all_to_all_single(a2a, torch.arange(P * 2, dtype=torch.int64) + 100 * r)
        res.append(a2a.tolist())
        nxt, prv = (r + 1) % P, (r - 1) % P
        got = torch.empty(4)
        comm.sendrecv({nxt: torch.full((4,), float(r))}, {prv: got})
        res.append(got.tolist())
        g1, g2 = torch.empty(2), torch.empty(3, dtype=torch.int64)
        comm.sendrecv_multi({nxt: [torch.full((2,), 7.0 + r), torch.arange(3) + r]}, {prv: [g1, g2]})
        res.append((g1.tolist(), g2.tolist()))
        out[ds] = res
    comm.dev_stage = False
    return out


def test_nccl_host_tensor_staging_matches_direct():
    for o in launch(_dev_stage_worker, 3, timeout=300):
        assert o[False] == o[True]


def _int16_wire_worker(comm):
    """RCCL has no int16 type (ShortArray tables): under nccl, data movement sends the bits
    as float16 and reductions run on an int32 copy. Forced here on gloo CPU ranks (the
    device-copy path switched off, so the wire-type path itself runs)."""
    comm.dev_stage = True
    comm._on_host = lambda *ts: False
    P, r = comm.world_size, comm.rank
    res = {}
    t = torch.tensor([30000, -30000, 7 + r, -1], dtype=torch.int16)
    a = t.clone()
    comm.all_reduce(a, op=torch.distributed.ReduceOp.MAX)
    res["max"] = a.tolist()
    s = torch.tensor([1000 * (r + 1), -5], dtype=torch.int16)
    comm.all_reduce(s)
    res["sum"] = s.tolist()
    b = torch.tensor([-32768, 32767, r, 0x7C01 - 65536 * 0], dtype=torch.int16)  # NaN bit pattern in fp16
    comm.broadcast(b, 1)
    res["bcast"] = b.tolist()
    g = torch.empty(2 * P, dtype=torch.int16)
    comm.all_gather_into(g, torch.tensor([-r - 1, 0x7E00 + r], dtype=torch.int16))
    res["gather"] = g.tolist()
    o = torch.empty(2, dtype=torch.int16)
    comm.reduce_scatter(o, torch.arange(2 * P, dtype=torch.int16) * (r + 1))
    res["rs"] = o.tolist()
    x = torch.empty(P, dtype=torch.int16)
    comm.all_to_all_single(x, (torch.arange(P, dtype=torch.int16) - 100 * r))
    res["a2a"] = x.tolist()
    rv = torch.empty(3, dtype=torch.int16)
    comm.sendrecv({(r + 1) % P: torch.tensor([r, -r, 0x7C01], dtype=torch.int16)}, {(r - 1) % P: rv})
    res["ring"] = rv.tolist()
    return res


def test_int16_tables_travel_bit_exact_on_the_rccl_wire_path():
    P = 2
    out = launch(_int16_wire_worker, P, timeout=300)
    for r, o in enumerate(out):
        assert o["max"] == [30000, -30000, 7 + P - 1, -1]
        assert o["sum"] == [1000 * P * (P + 1) // 2, -5 * P]
        assert o["bcast"] == [-32768, 32767, 1, 0x7C01]
        assert o["gather"] == [v for q in range(P) for v in (-q - 1, 0x7E00 + q)]
        assert o["rs"] == [(2 * r + j) * P * (P + 1) // 2 for j in range(2)]
        assert o["a2a"] == [r - 100 * q for q in range(P)]
        q = (r - 1) % P
        assert o["ring"] == [q, -q, 0x7C01]
