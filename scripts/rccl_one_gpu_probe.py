"""Probe: can two ranks on ONE MI355X form an RCCL ("nccl") process group?

The pool's boxes have one GPU, so every multi-rank path so far ran over gloo. RCCL normally
refuses two ranks on one device (duplicate bus id); this probe records what this image's
RCCL does, and if the group forms, runs the collectives the framework's Communicator uses
(all_reduce, all_gather_into_tensor, reduce_scatter_tensor, all_to_all_single, broadcast,
grouped send/recv ring) and checks every result.

Run: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
     --master-port 29511 scripts/rccl_one_gpu_probe.py
"""
from __future__ import annotations

import datetime
import os
import sys

import torch
import torch.distributed as dist


def main() -> int:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", timeout=datetime.timedelta(seconds=60), device_id=dev)
    ok = True

    def check(name, got, want):
        nonlocal ok
        good = torch.equal(got.cpu(), want.cpu())
        ok &= good
        print(f"rank {rank}: {name} {'ok' if good else 'MISMATCH'}", flush=True)

    x = torch.full((1 << 20,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    check("all_reduce", x, torch.full_like(x, world * (world + 1) / 2))
    y = torch.arange(8, device=dev, dtype=torch.float32) + 100 * rank
    g = torch.empty(world * 8, device=dev)
    dist.all_gather_into_tensor(g, y)
    check("all_gather", g, torch.cat([torch.arange(8, dtype=torch.float32) + 100 * r for r in range(world)]))
    z = torch.arange(world * 4, device=dev, dtype=torch.float32) * (rank + 1)
    rs = torch.empty(4, device=dev)
    dist.reduce_scatter_tensor(rs, z)
    check("reduce_scatter", rs, (torch.arange(world * 4, dtype=torch.float32) * world * (world + 1) / 2)[rank * 4:(rank + 1) * 4])
    a = torch.arange(world * 3, device=dev, dtype=torch.float32) + 1000 * rank
    b = torch.empty_like(a)
    dist.all_to_all_single(b, a)
    check("all_to_all", b, torch.cat([torch.arange(rank * 3, rank * 3 + 3, dtype=torch.float32) + 1000 * r
                                      for r in range(world)]))
    c = torch.full((16,), float(rank), device=dev)
    dist.broadcast(c, 0)
    check("broadcast", c, torch.zeros(16))
    s = torch.full((1024,), float(rank), device=dev)
    r_ = torch.empty_like(s)
    ops = [dist.P2POp(dist.isend, s, (rank + 1) % world), dist.P2POp(dist.irecv, r_, (rank - 1) % world)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    check("ring send/recv", r_, torch.full((1024,), float((rank - 1) % world)))
    torch.cuda.synchronize()
    dist.barrier()
    print(f"rank {rank}: RCCL world={world} on one GPU: {'PASS' if ok else 'FAIL'}", flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
