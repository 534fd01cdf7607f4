"""Device test utilities (``csrc/testutil.hip``): a bounded CU hog for rehearsing the
cooperative kernels under CU contention on one GPU."""
from __future__ import annotations

import torch

from . import _lib

_lib.register({"harp_test_spin": [_lib.c_int, _lib.c_int, _lib.c_long, _lib.c_void_p, _lib.c_void_p]})


def cu_hog(blocks: int, lds_bytes: int, us: int, stream: torch.cuda.Stream) -> torch.Tensor:
    """Launch ``blocks`` 256-thread workgroups on ``stream``, each holding ``lds_bytes`` of
    LDS for ``us`` microseconds; returns the (device) count of finished workgroups."""
    done = torch.zeros(1, dtype=torch.int32, device=stream.device)
    _lib.check(_lib.kernels().harp_test_spin(blocks, lds_bytes, us, done.data_ptr(), stream.cuda_stream), "test_spin")
    return done
