"""The reference's MF-SGD accuracy gate on its own ML-10M split, on any device.

ml/java/test_scripts/mfsgd.sh:64 -- SGDLauncher <train> 40 0.05 0.002 200 100 2 16 ...:
r = 40, lambda = 0.05, epsilon = 0.002, 200 iterations, trainRatio 100 (every rating every
iteration), 2 workers; pass if the final test RMSE is in (0.80, 0.84) (reference run 0.8345).
Data: /root/reference/datasets/daal_als/movielens-{train,test} (read-only text files).

    python scripts/ml10m_gate.py --device cuda --workers 2   # 2 gloo ranks sharing one GPU
    python scripts/ml10m_gate.py --device cpu --workers 2 --threads 4

On the GPU the factors are stored at the next kernel rank (48) with zero columns
(ops.mf.kernel_rank: exact). Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DATA = "/root/reference/datasets/daal_als"
PACKED = os.path.join(ROOT, "data", "ml10m", "ml10m.npz")  # u int32, i uint16, 2 x rating uint8


def job(comm, cfg, nu, ni, train, test, device):
    import torch

    from harp_amd.models.sgd_mf import SGDCollectiveMapper
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    if device == "cuda":
        comm = Communicator(None, torch.device("cuda", 0))
    m = SGDCollectiveMapper(comm, cfg, nu, ni, train, test)
    t0 = time.perf_counter()
    m.run(KeyValReader([]))
    wall = time.perf_counter() - t0
    res = m.result
    return {"rmse": res["rmse"], "trained": res["trained"], "epoch_s": res["epoch_s"], "wall_s": wall,
            "placement": res["placement"], "storage_rank": int(m.W.shape[1]), "blocks_per_xcd": m.bpx,
            "hot_items": m.hot_items, "atomic": m.atomic}


def als_job(comm, cfg, nu, ni, train, test, device):
    import torch

    from harp_amd.models.als import train_als
    from harp_amd.parallel.comm import Communicator

    if device == "cuda":
        comm = Communicator(None, torch.device("cuda", 0))
    P, me = comm.world_size, comm.rank
    u, i, v = train
    mine = torch.arange(u.numel()) % P == me  # any split of the training triples (train_als shuffles)
    t0 = time.perf_counter()
    r = train_als(comm, u[mine], i[mine], v[mine], nu, ni, cfg, test=test)
    return {"history": r["history"], "wall_s": time.perf_counter() - t0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu", choices=("cpu", "cuda"))
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--threads", type=int, default=4, help="CPU BlockScheduler threads per worker")
    ap.add_argument("--epochs", type=int, default=200)
    ap.add_argument("--rank", type=int, default=40)
    ap.add_argument("--atomic", type=int, default=-1, help="GPU: atomic write-back 0 none / 1 W / 2 H / 3 both (-1 = model default)")
    ap.add_argument("--blocks-per-xcd", type=int, default=0)
    ap.add_argument("--conflict-mode", default="hot", help="GPU: hot (lossless hot items, full concurrency) / cap / none")
    ap.add_argument("--hot-residual", type=float, default=-1.0)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--als", action="store_true",
                    help="DAAL implicit ALS instead (harp-daal-als.sh:51-63: Dim 100, lambda 0.05, 5 iterations)")
    ap.add_argument("--pack", action="store_true", help=f"write {PACKED} from the reference text files and exit")
    args = ap.parse_args()
    if args.pack:
        import numpy as np

        from harp_amd.utils.datasets import load_coo

        arrs = {}
        for name in ("train", "test"):
            u, i, v = load_coo(os.path.join(DATA, "movielens-" + name), sep=" ")
            assert int(i.max()) < 65535 and bool(((v * 2).round() == v * 2).all())
            arrs[name + "_u"] = u.numpy().astype(np.int32)
            arrs[name + "_i"] = i.numpy().astype(np.uint16)
            arrs[name + "_v2"] = (v * 2).round().numpy().astype(np.uint8)
        os.makedirs(os.path.dirname(PACKED), exist_ok=True)
        np.savez_compressed(PACKED, **arrs)
        return

    from harp_amd.models.sgd_mf import SGDConfig
    from harp_amd.runtime.launcher import launch
    from harp_amd.utils.datasets import load_coo

    t0 = time.perf_counter()
    if os.path.isdir(DATA):
        u, i, v = load_coo(os.path.join(DATA, "movielens-train"), sep=" ")
        tu, ti, tv = load_coo(os.path.join(DATA, "movielens-test"), sep=" ")
        src = DATA
    else:  # the GPU box has no reference checkout: the same split packed by this script (--pack)
        import numpy as np
        import torch

        z = np.load(PACKED)  # plain arrays, allow_pickle=False
        col = lambda k, dt: torch.from_numpy(z[k].astype(dt))  # noqa: E731
        u, i, v = col("train_u", np.int64), col("train_i", np.int64), col("train_v2", np.float32) / 2
        tu, ti, tv = col("test_u", np.int64), col("test_i", np.int64), col("test_v2", np.float32) / 2
        src = PACKED
    load_s = time.perf_counter() - t0
    nu, ni = int(max(u.max(), tu.max())) + 1, int(max(i.max(), ti.max())) + 1
    if args.als:
        from harp_amd.models.als import ALSConfig

        acfg = ALSConfig(factors=100, lam=0.05, alpha=40.0, iterations=5, implicit=True)
        res = launch(als_job, args.workers, args=(acfg, nu, ni, (u, i, v.double()), (tu, ti, tv.double()), args.device),
                     timeout=1100)
        h = res[0]["history"]
        print(json.dumps({"app": "daal_als (harp-daal-als.sh:51-63)", "data": src, "device": args.device,
                          "workers": args.workers, "factors": 100, "lambda": 0.05, "alpha": 40.0, "iterations": 5,
                          "test_conf_rmse": h[-1].get("test_conf_rmse"), "test_rmse_vs_ratings": h[-1]["test_rmse"],
                          "history": h, "wall_s": max(r["wall_s"] for r in res)}))
        return
    cfg = SGDConfig(rank=args.rank, lam=0.05, lr=0.002, epochs=args.epochs, num_slices=2, test_every=5,
                    init="reference", cpu_threads=args.threads if args.device == "cpu" else 1, chunk=args.chunk)
    if args.atomic >= 0:
        cfg.atomic = args.atomic
    if args.blocks_per_xcd:
        cfg.blocks_per_xcd = args.blocks_per_xcd
    if args.conflict_mode:
        cfg.conflict_mode = args.conflict_mode
    if args.hot_residual >= 0:
        cfg.hot_residual = args.hot_residual
    res = launch(job, args.workers, args=(cfg, nu, ni, (u, i, v.float()), (tu, ti, tv.float()), args.device),
                 timeout=1100)
    r0 = res[0]
    test_rmse = r0["rmse"][-1][2]
    out = {
        "gate": "mfsgd.sh:64 r=40 lambda=0.05 eps=0.002 200 iters 2 workers, test RMSE in (0.80, 0.84)",
        "data": src, "device": args.device, "atomic": r0.get("atomic", cfg.atomic), "blocks_per_xcd": r0["blocks_per_xcd"],
        "conflict_mode": cfg.conflict_mode, "hot_residual": cfg.hot_residual, "hot_items": r0.get("hot_items"),
        "chunk": cfg.chunk, "workers": args.workers, "rank": args.rank, "storage_rank": r0["storage_rank"],
        "train_ratings": int(u.numel()), "test_ratings": int(tu.numel()),
        "test_rmse": test_rmse, "pass": 0.80 < test_rmse < 0.84, "reference_run": 0.8345,
        "trained": sum(r["trained"] for r in res),
        "mean_epoch_s": max(sum(r["epoch_s"]) / len(r["epoch_s"]) for r in res),
        "wall_s": max(r["wall_s"] for r in res), "load_s": load_s,
        "placement": [r["placement"] for r in res],
        "rmse_curve": r0["rmse"],
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
