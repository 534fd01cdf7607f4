"""Partition combiners (Harp L2).

Reference semantics:
  * ``PartitionCombiner.combine(cur, new) -> PartitionStatus`` merges ``new`` into
    ``cur`` in place (core/harp-collective/.../partition/PartitionCombiner.java:36).
  * ``PartitionStatus`` = ADDED / ADD_FAILED / COMBINED / COMBINE_FAILED
    (partition/PartitionStatus.java:22-24).
  * typed array combiners apply SUM / MINUS / MULTIPLY / MAX / MIN element-wise and
    fail when the sizes differ (combiner/DoubleArrCombiner.java:24-68; Int/Long/Short/
    Byte variants are identical up to the element type).

MI355X design: payloads are ``torch.Tensor`` (CPU or HIP device) so a combine is one
in-place device op; for packed tables the collectives never call these at all — the
combine happens inside RCCL's reduction (``Operation.rccl_op``).
"""
from __future__ import annotations

import enum
from typing import Any

import torch


class PartitionStatus(enum.Enum):
    ADDED = 0
    ADD_FAILED = 1
    COMBINED = 2
    COMBINE_FAILED = 3


class Operation(enum.Enum):
    SUM = "sum"
    MINUS = "minus"
    MULTIPLY = "multiply"
    MAX = "max"
    MIN = "min"

    @property
    def rccl_op(self):
        """The torch.distributed ReduceOp that implements this combine inside a
        collective, or None when the op is order dependent (MINUS)."""
        import torch.distributed as dist

        return {
            Operation.SUM: dist.ReduceOp.SUM,
            Operation.MULTIPLY: dist.ReduceOp.PRODUCT,
            Operation.MAX: dist.ReduceOp.MAX,
            Operation.MIN: dist.ReduceOp.MIN,
        }.get(self)


class PartitionCombiner:
    """Base combiner. Subclasses override :meth:`combine`."""

    #: Operation used by the dense fast path when every partition is a tensor.
    #: ``None`` forces the generic (host-ordered) combine path.
    operation: Operation | None = None

    def combine(self, cur: Any, new: Any) -> PartitionStatus:  # pragma: no cover - abstract
        raise NotImplementedError

    def __repr__(self) -> str:
        return f"{type(self).__name__}({self.operation})"


def _payload_tensor(x: Any) -> torch.Tensor | None:
    if isinstance(x, torch.Tensor):
        return x
    t = getattr(x, "tensor", None)
    if isinstance(t, torch.Tensor):
        return t
    return None


def combine_tensors(op: Operation, cur: torch.Tensor, new: torch.Tensor) -> PartitionStatus:
    if cur.numel() != new.numel():
        return PartitionStatus.COMBINE_FAILED
    if new.device != cur.device or new.dtype != cur.dtype:
        new = new.to(device=cur.device, dtype=cur.dtype)
    if new.shape != cur.shape:
        new = new.reshape(cur.shape)
    if op is Operation.SUM:
        cur.add_(new)
    elif op is Operation.MINUS:
        cur.sub_(new)
    elif op is Operation.MULTIPLY:
        cur.mul_(new)
    elif op is Operation.MAX:
        torch.maximum(cur, new, out=cur)
    elif op is Operation.MIN:
        torch.minimum(cur, new, out=cur)
    else:  # pragma: no cover
        return PartitionStatus.COMBINE_FAILED
    return PartitionStatus.COMBINED


class ArrCombiner(PartitionCombiner):
    """Element-wise combiner for any typed array / tensor payload.

    One class replaces the reference's Byte/Short/Int/Long/Double ArrCombiner family
    (combiner/*ArrCombiner.java); the element type is the tensor's dtype.
    """

    def __init__(self, operation: Operation = Operation.SUM):
        self.operation = Operation(operation)

    def combine(self, cur: Any, new: Any) -> PartitionStatus:
        a, b = _payload_tensor(cur), _payload_tensor(new)
        if a is None or b is None:
            return PartitionStatus.COMBINE_FAILED
        return combine_tensors(self.operation, a, b)


# Named aliases matching the reference's typed combiners / example combiners
# (combiner/DoubleArrCombiner.java, example/DoubleArrPlus.java, IntArrPlus.java, LongArrPlus.java).
class DoubleArrCombiner(ArrCombiner):
    pass


class FloatArrCombiner(ArrCombiner):
    pass


class IntArrCombiner(ArrCombiner):
    pass


class LongArrCombiner(ArrCombiner):
    pass


class ShortArrCombiner(ArrCombiner):
    pass


class ByteArrCombiner(ArrCombiner):
    pass


class DoubleArrPlus(ArrCombiner):
    def __init__(self):
        super().__init__(Operation.SUM)


class IntArrPlus(ArrCombiner):
    def __init__(self):
        super().__init__(Operation.SUM)


class LongArrPlus(ArrCombiner):
    def __init__(self):
        super().__init__(Operation.SUM)


class FloatArrPlus(ArrCombiner):
    def __init__(self):
        super().__init__(Operation.SUM)


class ArrMax(ArrCombiner):
    """(harp-daal-interface data_aux/IntArrMax.java, LongArrMax.java)"""

    def __init__(self):
        super().__init__(Operation.MAX)


class ArrMin(ArrCombiner):
    def __init__(self):
        super().__init__(Operation.MIN)


class WritableCombiner(PartitionCombiner):
    """Delegates to ``cur.combine(new)`` for user Writable payloads that define it."""

    def combine(self, cur: Any, new: Any) -> PartitionStatus:
        fn = getattr(cur, "combine", None)
        if fn is None:
            return PartitionStatus.COMBINE_FAILED
        res = fn(new)
        return res if isinstance(res, PartitionStatus) else PartitionStatus.COMBINED


class NoCombine(PartitionCombiner):
    """Keeps the existing partition (first writer wins)."""

    def combine(self, cur: Any, new: Any) -> PartitionStatus:
        return PartitionStatus.COMBINED


class ReplaceCombiner(PartitionCombiner):
    """Overwrites the current payload in place with the new one (last writer wins)."""

    def combine(self, cur: Any, new: Any) -> PartitionStatus:
        a, b = _payload_tensor(cur), _payload_tensor(new)
        if a is None or b is None or a.numel() != b.numel():
            return PartitionStatus.COMBINE_FAILED
        a.copy_(b.reshape(a.shape))
        return PartitionStatus.COMBINED
