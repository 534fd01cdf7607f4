"""The Harp K-means tutorial, written against the harp_amd API.

It ports `website/content/docs/examples/kmeans.md` from the reference (allreduce,
broadcast-reduce, push-pull and regroup-allgather, the four `runKmeans` variants) as
user code. A subclass of `CollectiveMapper` keeps a centroid `Table` of one partition per
centroid. The last slot of each partition is the point count, combined with
`DoubleArrPlus`. The four strategies synchronise it with the Harp collectives named by
(context, operation).

The production K-means is `harp_amd.models.kmeans` (MFMA assign kernel, packed tables,
cached plans). This file shows that the programming model carries over line for line.

Run it with two local workers:

    python examples/kmeans_tutorial.py --workers 2 --strategy allreduce

or one process per GPU under torchrun:

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m harp_amd.runtime.launcher \\
        --mapper examples.kmeans_tutorial:KMeansTutorialMapper --conf '{"strategy": "allreduce"}'
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from harp_amd.core import DoubleArrPlus, Partitioner, Table  # noqa: E402
from harp_amd.runtime.mapper import CollectiveMapper, Context, KeyValReader  # noqa: E402


class KMeansTutorialMapper(CollectiveMapper):
    """The tutorial's mapper. ``context.conf`` holds: n (points per worker), k, d,
    iterations, strategy, seed."""

    def map_collective(self, reader: KeyValReader, context: Context) -> None:
        conf = context.get_configuration()
        n, k, d = int(conf.get("n", 1000)), int(conf.get("k", 10)), int(conf.get("d", 10))
        iters, strategy = int(conf.get("iterations", 10)), conf.get("strategy", "allreduce")
        seed = int(conf.get("seed", 0))
        dev = self.device
        # this worker's points (the tutorial loads its point files; synthetic here)
        g = torch.Generator().manual_seed(seed * 1000 + self.get_self_id())
        points = (torch.rand((n, d), generator=g, dtype=torch.float64) * 10).to(dev)

        # master loads the initial centroids, then broadcasts them (loadCentroids + broadcastCentroids)
        cen = Table(0, DoubleArrPlus())
        if self.is_master():
            g0 = torch.Generator().manual_seed(seed)
            for c in range(k):
                row = torch.zeros(d + 1, dtype=torch.float64)
                row[:d] = torch.rand(d, generator=g0, dtype=torch.float64) * 10
                cen.add(c, row.to(dev))
        if not self.broadcast("main", "broadcast-centroids", cen, 0, use_mst=False):
            raise IOError("broadcast failed")

        for it in range(iters):
            prev = cen
            cen = Table(0, DoubleArrPlus())
            self.computation(cen, prev, points)  # local partial sums (last slot = count)
            if strategy == "allreduce":
                self.allreduce("main", f"allreduce_{it}", cen)
                self.calculate_centroids(cen)
            elif strategy == "broadcast-reduce":
                self.reduce("main", f"reduce_{it}", cen, 0)
                if self.is_master():
                    self.calculate_centroids(cen)
                else:
                    cen = Table(0, DoubleArrPlus())
                self.broadcast("main", f"bcast_{it}", cen, 0, use_mst=True)
            elif strategy == "push-pull":
                # the global table is distributed over the workers (owner = id % P)
                glob = Table(1, DoubleArrPlus())
                self.push("main", f"push_{it}", cen, glob, Partitioner(self.get_num_workers()))
                self.calculate_centroids(glob)
                for p in cen:
                    p.get().zero_()  # pull combines into the local partitions
                self.pull("main", f"pull_{it}", cen, glob, True)
            elif strategy == "regroup-allgather":
                self.regroup("main", f"regroup_{it}", cen, Partitioner(self.get_num_workers()))
                self.calculate_centroids(cen)
                self.allgather("main", f"allgather_{it}", cen)
            else:
                raise ValueError(f"unknown strategy {strategy}")
        # mean point -> nearest centroid distance (the quantity of the reference's km.sh gate)
        C = torch.stack([cen[i][:d] for i in cen.sorted_ids()])
        self.result = {"centroids": C.cpu(), "mean_distance": float(torch.cdist(points, C).min(1).values.mean())}

    @staticmethod
    def computation(cen: Table, prev: Table, points: torch.Tensor) -> None:
        ids = prev.sorted_ids()
        d = points.shape[1]
        C = torch.stack([prev[i][:d] for i in ids])
        lab = torch.cdist(points, C).argmin(1)
        sums = torch.zeros((len(ids), d + 1), dtype=points.dtype, device=points.device)
        sums[:, :d].index_add_(0, lab, points)
        sums[:, d] = torch.bincount(lab, minlength=len(ids)).to(points.dtype)
        for j, i in enumerate(ids):
            cen.add(i, sums[j].clone())

    @staticmethod
    def calculate_centroids(cen: Table) -> None:
        for p in cen:
            row = p.get()
            if row[-1] > 0:
                row[:-1] /= row[-1]
                row[-1] = 0.0  # the count slot restarts at zero for the next combine


def _job(comm, conf):
    from harp_amd.runtime.launcher import run_mapper

    return run_mapper(comm, KMeansTutorialMapper, [], conf)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--strategy", default="allreduce",
                    choices=["allreduce", "broadcast-reduce", "push-pull", "regroup-allgather"])
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--d", type=int, default=10)
    ap.add_argument("--iterations", type=int, default=10)
    a = ap.parse_args(argv)
    from harp_amd.runtime.launcher import launch

    conf = {"n": a.n, "k": a.k, "d": a.d, "iterations": a.iterations, "strategy": a.strategy}
    res = launch(_job, a.workers, args=(conf,), timeout=300)
    print(json.dumps({"strategy": a.strategy, "mean_distance": [r["mean_distance"] for r in res],
                      "centroid0": [round(float(x), 4) for x in res[0]["centroids"][0]]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
