"""harp_amd — an MI355X-native collective-communication framework for iterative ML.

Capabilities of Harp (chathurawidanage/harp) re-designed for MI355X: key-addressed
partition tables and Harp's collectives (broadcast, reduce, allgather, allreduce,
regroup/aggregate, push/pull, rotate, join, barrier, events) over RCCL/xGMI, hand-written
gfx950 HIP kernels for the workloads' hot loops, and the CollectiveMapper programming
model.
"""
__version__ = "0.1.0"

from .core import *  # noqa: F401,F403
