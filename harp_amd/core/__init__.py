from .arrays import (Array, ByteArray, DoubleArray, FloatArray, IntArray, LongArray,  # noqa: F401
                     ShortArray)
from .combiner import (ArrCombiner, ByteArrCombiner, DoubleArrCombiner, DoubleArrPlus,  # noqa: F401
                       FloatArrCombiner, IntArrCombiner, IntArrPlus, LongArrCombiner, LongArrPlus,
                       Operation, PartitionCombiner, PartitionStatus, ShortArrCombiner)
from .partition import (UNKNOWN_WORKER_ID, MapPartitioner, Partition, PartitionFunction,  # noqa: F401
                        Partitioner, RandomPartitioner)
from .pool import ArrayPool, ResourcePool  # noqa: F401
from .table import PackedTable, Table  # noqa: F401
from .writable import DataInput, DataOutput, Writable, register_writable  # noqa: F401
