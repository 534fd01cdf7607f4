"""Multi-host driver: nodes-file planning and a real local 2-node x 1-proc run (gloo)."""
import json
import os
import sys

from harp_amd.runtime import driver as D


def test_plan_ranks_and_master():
    text = "#0\nhostA\nhostB\n#1\nhostC\n"
    pl = D.plan(text, ["-m", "harp_amd.examples", "--op", "allreduce"], 8)
    assert [p.host for p in pl] == ["hostA", "hostB", "hostC"]
    assert all("--master-addr=hostA" in p.argv for p in pl)
    assert [p.argv[p.argv.index("--nnodes=3") + 1] for p in pl] == ["--node-rank=0", "--node-rank=1", "--node-rank=2"]
    cmd = D._command(pl[1], ())
    assert cmd[0] == "ssh" and cmd[3] == "hostB"


def test_local_two_node_job(tmp_path):
    text = "#0\n127.0.0.1\nlocalhost\n"
    port = 29000 + os.getpid() % 1000
    pl = D.plan(text, ["-m", "harp_amd.examples", "--backend", "gloo", "--op", "allgather", "--elements", "8",
                       "--iterations", "2", "--verify"], 1, master_port=port, log_dir=str(tmp_path))
    codes = D.run(pl, timeout_s=240)
    assert codes == [0, 0], [open(p.log).read()[-2000:] for p in pl]
    out = open(pl[0].log).read()
    line = [ln for ln in out.splitlines() if ln.startswith("{")][-1]
    r = json.loads(line)
    assert r["workers"] == 2 and r["verified_partitions"] == 4  # 2 iterations x 2 partitions
