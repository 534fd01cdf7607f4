"""Collective examples with --verify (ExamplesMain: allreduce / allgather / reduce /
bcast / rotate, plus regroup and push/pull) on 3 gloo workers, packed and generic
tables, several data types; and the CLI entry point."""
import json
import subprocess
import sys

import pytest

from harp_amd.examples import OPS, run_example
from harp_amd.runtime.launcher import launch


@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("packed", [True, False])
def test_example_verifies(op, packed):
    conf = {"op": op, "elements": 64, "partitions": 3, "iterations": 4, "data_type": "double", "verify": True,
            "packed": packed}
    res = launch(run_example, 3, args=(conf,), timeout=300)
    assert all(r["verify"] for r in res)
    assert sum(r["verified_partitions"] for r in res) > 0


@pytest.mark.parametrize("dtype", ["int", "float", "long"])
def test_example_dtypes(dtype):
    conf = {"op": "allreduce", "elements": 16, "partitions": 2, "iterations": 3, "data_type": dtype, "verify": True}
    res = launch(run_example, 2, args=(conf,), timeout=300)
    assert res[0]["verified_partitions"] == 6


def test_examples_cli():
    out = subprocess.run([sys.executable, "-m", "harp_amd.examples", "--spawn", "2", "--op", "allgather",
                          "--elements", "32", "--iterations", "2", "--verify"], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    r = json.loads(line)
    assert r["op"] == "allgather" and r["workers"] == 2 and r["verified_partitions"] == 2 * 2
