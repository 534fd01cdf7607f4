"""Multi-host job driver (the non-Hadoop ``Driver`` + MapCollective launcher role).

Reference: core/harp-collective/.../collective/Driver.java:183-268 (read the nodes file,
``ssh host script driverHost driverPort workerID jobID args &`` per worker, wait for P
``report-to-driver`` acks, per-worker log ``harp-worker-<id>.log``) and the YARN
MapCollectiveContainerLauncherImpl (writes ``nodes`` / ``tasks`` files, gang-schedules
all mappers).

MI355X design: a host runs ONE torchrun per node with ``--nproc-per-node`` = its GPU
count (one process per GPU, RCCL over xGMI inside the node); the driver only builds the
per-host command lines from the nodes file (rack order = rank order, like
Workers.java), starts them (locally via subprocess, remotely via ssh), streams each
node's output into ``harp-node-<n>.log`` and returns the exit codes. Rendezvous is
torch.distributed's (``--master-addr`` = first host), replacing the lock-file poll.
"""
from __future__ import annotations

import argparse
import os
import shlex
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

from ..parallel.comm import parse_nodes_file

LOCAL = {"localhost", "127.0.0.1", "::1"}


@dataclass
class NodeLaunch:
    node_rank: int
    host: str
    argv: List[str]
    log: str


def plan(nodes_text: str, module_argv: Sequence[str], nproc_per_node: int, master_port: int = 29500,
         log_dir: str = ".", python: str = sys.executable) -> List[NodeLaunch]:
    """One torchrun command per host in nodes-file order (racks concatenated)."""
    hosts = [h for rack in parse_nodes_file(nodes_text) for h in rack]
    if not hosts:
        raise ValueError("nodes file lists no hosts")
    master = "127.0.0.1" if hosts[0] in LOCAL else hosts[0]
    out = []
    for n, h in enumerate(hosts):
        argv = [python, "-m", "torch.distributed.run", f"--nnodes={len(hosts)}", f"--node-rank={n}",
                f"--nproc-per-node={nproc_per_node}", f"--master-addr={master}", f"--master-port={master_port}",
                *module_argv]
        out.append(NodeLaunch(n, h, argv, os.path.join(log_dir, f"harp-node-{n}.log")))
    return out


def _command(nl: NodeLaunch, env_keep: Sequence[str]) -> List[str]:
    if nl.host in LOCAL:
        return nl.argv
    exports = " ".join(f"{k}={shlex.quote(os.environ[k])}" for k in env_keep if k in os.environ)
    remote = f"cd {shlex.quote(os.getcwd())} && {exports} {' '.join(shlex.quote(a) for a in nl.argv)}"
    return ["ssh", "-o", "BatchMode=yes", nl.host, remote]


def run(launches: List[NodeLaunch], timeout_s: float = 24 * 3600,
        env_keep: Sequence[str] = ("HSA_ENABLE_IPC_MODE_LEGACY", "PYTHONPATH")) -> List[int]:
    """Start every node, wait for all (or the timeout), return the exit codes."""
    procs = []
    for nl in launches:
        os.makedirs(os.path.dirname(nl.log) or ".", exist_ok=True)
        fh = open(nl.log, "w")
        procs.append((subprocess.Popen(_command(nl, env_keep), stdout=fh, stderr=subprocess.STDOUT), fh))
    deadline = time.monotonic() + timeout_s
    codes: List[Optional[int]] = [None] * len(procs)
    while any(c is None for c in codes):
        for i, (p, _) in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        if any(c not in (None, 0) for c in codes):
            break  # one node failed: stop the job (fail-fast, like a lost mapper)
        if time.monotonic() > deadline:
            break
        time.sleep(0.2)
    for i, (p, fh) in enumerate(procs):
        if codes[i] is None:
            p.terminate()
            try:
                codes[i] = p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
                codes[i] = p.wait()
        fh.close()
    return [int(c) for c in codes]


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="Launch a harp_amd job on the hosts of a Harp nodes file")
    ap.add_argument("--nodes", required=True, help="nodes file (#rack lines + hostnames)")
    ap.add_argument("--nproc-per-node", type=int, default=8)
    ap.add_argument("--master-port", type=int, default=29500)
    ap.add_argument("--log-dir", default=".")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("rest", nargs=argparse.REMAINDER, help="-- module/script and its args")
    a = ap.parse_args(argv)
    rest = a.rest[1:] if a.rest and a.rest[0] == "--" else a.rest
    with open(a.nodes) as f:
        launches = plan(f.read(), rest, a.nproc_per_node, a.master_port, a.log_dir)
    if a.dry_run:
        for nl in launches:
            print(nl.host, " ".join(shlex.quote(x) for x in _command(nl, ())))
        return 0
    codes = run(launches)
    print("exit codes:", codes)
    return max(codes) if codes else 0


if __name__ == "__main__":
    sys.exit(main())
