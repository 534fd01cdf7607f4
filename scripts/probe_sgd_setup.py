"""Profile of the MF-SGD record's setup (synthetic ratings + init_model) on P gloo ranks that
share one GPU: python scripts/probe_sgd_setup.py P"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def run(rank, P, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    dist.init_process_group("gloo", rank=rank, world_size=P)
    import cProfile
    import pstats

    from harp_amd.models.sgd_mf import SGDCollectiveMapper, SGDConfig, synthetic_ratings
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    comm = Communicator(None, dev)
    t0 = time.perf_counter()
    u, i, v = synthetic_ratings(480189, 17770, 100480507, seed=7, device=dev)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    cfg = SGDConfig(rank=128, epochs=2, test_every=0, xcd_blocks=dev.type == "cuda", num_slices=1)
    m = SGDCollectiveMapper(comm, cfg, 480189, 17770, (u, i, v), None)
    pr = cProfile.Profile()
    pr.enable()
    m.init_model(KeyValReader([]))
    torch.cuda.synchronize()
    pr.disable()
    t2 = time.perf_counter()
    print(f"rank {rank}: ratings {t1 - t0:.2f}s init {t2 - t1:.2f}s", flush=True)
    if rank == 0:
        pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
    dist.destroy_process_group()


if __name__ == "__main__":
    P = int(sys.argv[1])
    mp.spawn(run, args=(P, 29741), nprocs=P)
