"""K-means under a modelled SGX-enclave cost (experimental ``kmeans/sgxsimu``).

Reference: experimental/src/main/java/edu/iu/kmeans/sgxsimu/ —
KMeansCollectiveMapper.java:155-384 runs regroup-allgather K-means and, when simulation
is on, *sleeps* for the modelled cost of every enclave transition: enclave creation and
local attestation once (:172-197), an ecall per point shard copied into a thread enclave
plus an EPC-paging "memory" term proportional to the measured compute time
(CenCalcTask.java:127-195, ``sgx_overhead_func`` :203-213), ecall+ocall for each thread's
centroid copy (CenCalcTask.java:73-83), and a cross-enclave transfer for the regroup
(:288-302) and the allgather (:333-345). The constants are kilo-cycles measured on an
SGX-enabled Xeon, converted at ``ms_per_kcycle`` (Constants.java:29-40).

Here the model is a pure function of the job shape (:class:`SGXCostModel`), applied on
top of the real MI355X K-means iteration (:class:`SGXKMeansMapper`): the GPU time is
measured with device synchronisation and the modelled enclave time is *accounted* per
phase (``sgx_*`` entries of the per-iteration record). ``sleep=True`` reproduces the
reference's behaviour of adding the modelled delay to wall-clock time.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from .kmeans import KMeansCollectiveMapper, KMeansConfig


@dataclass(frozen=True)
class SGXCostModel:
    """Enclave transition costs in kilo-cycles (Constants.java:31-40)."""

    ecall: float = 8.5
    ocall: float = 9.0
    cross_enclave_per_kb: float = 1.4
    creation_enclave_fix: float = 221000.0
    creation_enclave_kb: float = 22.677
    local_attestation: float = 80.0
    remote_attestation: float = 27200.0
    swap_page_penalty: float = 40.0
    ms_per_kcycle: float = 0.0002941  # 3.4 GHz part

    # the reference truncates every modelled delay to whole milliseconds (``(long)``)
    @staticmethod
    def _ms(x: float) -> int:
        return int(x)

    @staticmethod
    def double_kb(n_doubles: int) -> int:
        """KB of ``n`` doubles, integer-truncated like ``dataDoubleSizeKB``."""
        return n_doubles * 8 // 1024

    def enclave_creation_ms(self, enclave_total_mb: int, threads: int) -> int:
        per = (self.creation_enclave_fix + enclave_total_mb * 1024 * self.creation_enclave_kb) * self.ms_per_kcycle
        return self._ms(per * threads)

    def local_attestation_ms(self, threads: int, mappers: int) -> int:
        pairs = math.comb(threads, 2) + (mappers - 1) * threads
        return self._ms(pairs * self.local_attestation * self.ms_per_kcycle)

    def transfer_ms(self, kb: int, ecalls: int = 1, ocalls: int = 0) -> int:
        return self._ms((ecalls * self.ecall + ocalls * self.ocall + kb * self.cross_enclave_per_kb)
                        * self.ms_per_kcycle)

    def centroid_copy_ms(self, n_doubles: int) -> Dict[str, int]:
        """Per compute thread: ecall in + ocall out of its centroid copy."""
        kb = self.double_kb(n_doubles)
        return {"ecall": self.transfer_ms(kb, ecalls=1), "ocall": self.transfer_ms(kb, ecalls=0, ocalls=1)}

    @staticmethod
    def mem_ratio(shard_kb: int) -> float:
        """EPC paging slowdown fit of ``CenCalcTask.sgx_overhead_func`` (shard size in KB)."""
        s = shard_kb / 10.0 / 1024.0
        return -0.000592887941 * s ** 3 + 0.03776145898 * s ** 2 - 0.172624736 * s + 0.08813241271

    def shard_ms(self, shard_kb: int, compute_ms: float) -> Dict[str, int]:
        """One point shard through a thread enclave: ecall of the shard + paging term
        (proportional to the measured compute time, minus the ecall; clamped at 0)."""
        ecall = self.transfer_ms(shard_kb, ecalls=1)
        mem = max(0, self._ms(compute_ms * self.mem_ratio(shard_kb)) - ecall)
        return {"ecall": ecall, "mem": mem}

    def regroup_ms(self, table_kb: int, mappers: int) -> int:
        data = (table_kb // mappers) * (2 * mappers - 2)
        return self._ms((mappers - 1) * (self.ocall + self.ecall) * self.ms_per_kcycle
                        + data * self.cross_enclave_per_kb * self.ms_per_kcycle)

    def allgather_ms(self, table_kb: int, mappers: int) -> int:
        return self._ms((self.ocall + self.ecall * (mappers - 1)) * self.ms_per_kcycle
                        + table_kb * self.cross_enclave_per_kb * self.ms_per_kcycle)


@dataclass
class SGXConfig:
    enclave_total_mb: int = 96     # ENCLAVE_TOTAL
    enclave_per_thd_mb: int = 96   # ENCLAVE_PER_THD
    enclave_task_mb: int = 8       # ENCLAVE_TASK: size of one point shard (doubles)
    threads: int = 1               # enclaves per mapper (one per compute thread in the reference)
    enable: bool = True
    sleep: bool = False            # add the modelled delay to wall-clock time (reference behaviour)
    model: SGXCostModel = field(default_factory=SGXCostModel)


class SGXKMeansMapper(KMeansCollectiveMapper):
    """Regroup-allgather K-means whose iteration record carries the modelled enclave cost."""

    def __init__(self, comm=None, config: Optional[KMeansConfig] = None, sgx: Optional[SGXConfig] = None, **kw):
        config = config or KMeansConfig()
        config.strategy = "regroup_allgather"
        super().__init__(comm, config, **kw)
        self.sgx = sgx or SGXConfig()
        self.sgx_totals: Dict[str, float] = {"init": 0, "ecall": 0, "ocall": 0, "mem": 0, "comm": 0}
        self.sgx_iters: List[Dict[str, float]] = []

    def _delay(self, ms: float) -> None:
        if self.sgx.sleep and ms > 0:
            time.sleep(ms / 1e3)

    def init_model(self, reader) -> None:
        super().init_model(reader)
        s, m = self.sgx, self.sgx.model
        if s.enable:
            init = m.enclave_creation_ms(s.enclave_total_mb, s.threads) + \
                m.local_attestation_ms(s.threads, self.get_num_workers())
            self.sgx_totals["init"] += init
            self._delay(init)

    def _sync_device(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def step(self, it: int) -> None:
        if not self.sgx.enable:
            return super().step(it)
        s, m, cfg = self.sgx, self.sgx.model, self.cfg
        P = self.get_num_workers()
        self._sync_device()
        t0 = time.perf_counter()
        super().step(it)
        self._sync_device()
        compute_ms = (time.perf_counter() - t0) * 1e3
        # shards of ENCLAVE_TASK MB of doubles (shadSize, KMeansCollectiveMapper.java:114)
        n = self.X.shape[0]
        shard_pts = max(1, s.enclave_task_mb * 1024 * 1024 // (cfg.dim * 8))
        n_shards = math.ceil(n / shard_pts)
        shard_kb = m.double_kb(min(shard_pts, n) * cfg.dim)
        per = m.shard_ms(shard_kb, compute_ms / max(n_shards, 1))
        # shards are spread over the threads; the reference averages per-thread totals (:263-265)
        ecall = per["ecall"] * n_shards / s.threads
        mem = per["mem"] * n_shards / s.threads
        copy = m.centroid_copy_ms(cfg.num_centroids * (cfg.dim + 1))
        table_kb = m.double_kb(cfg.num_centroids * (cfg.dim + 1))
        comm = (m.regroup_ms(table_kb, P) + m.allgather_ms(table_kb, P)) if P > 1 else 0
        rec = {"iter": it, "gpu_ms": compute_ms, "ecall": ecall + copy["ecall"], "ocall": copy["ocall"],
               "mem": mem, "comm": comm}
        for k in ("ecall", "ocall", "mem", "comm"):
            self.sgx_totals[k] += rec[k]
        rec["sgx_ms"] = rec["ecall"] + rec["ocall"] + rec["mem"] + rec["comm"]
        self.sgx_iters.append(rec)
        self._delay(rec["sgx_ms"])

    def finish(self) -> None:
        super().finish()
        self.result["sgx"] = {"totals_ms": dict(self.sgx_totals), "iterations": list(self.sgx_iters)}


def run_sgx_kmeans(comm, cfg: KMeansConfig, sgx: Optional[SGXConfig] = None, points=None,
                   init_centroids=None) -> dict:
    """Launcher target: SGX-simulated K-means on this rank."""
    from ..runtime.mapper import KeyValReader

    m = SGXKMeansMapper(comm, cfg, sgx, points=points, init_centroids=init_centroids)
    m.run(KeyValReader([]))
    return {"objective": m.objective, "centroids": m.centroids.cpu(), "sgx": m.result["sgx"]}
