"""Per-collective golden tests on P gloo workers (SURVEY §7.3 phase 2 gate), including
odd P (the reference special-cases odd ranges, AllreduceCollective.java:175-180)."""
import pytest

from harp_amd.runtime.launcher import launch
from tests.mp_checks import collective_battery, runtime_battery


@pytest.mark.parametrize("P", [1, 2, 3, 4])
def test_collective_battery(P):
    results = launch(collective_battery, P, timeout=300)
    failures = {(rank, k): v for rank, res in enumerate(results) for k, v in res.items() if v is not True}
    assert not failures, failures


@pytest.mark.parametrize("P", [2, 3])
def test_runtime_battery(P):
    results = launch(runtime_battery, P, timeout=300)
    failures = {(rank, k): v for rank, res in enumerate(results) for k, v in res.items() if v is not True}
    assert not failures, failures
