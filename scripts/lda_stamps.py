#!/usr/bin/env python3
"""Per-phase clock totals of the dense LDA sampler (diagnostic build): runs
scripts/bench_lda.py with HARP_KERNEL_LIB pointing at a library built with
-DHARP_LDA_STAMPS (scripts/ab/liblda_stamps.so) and prints the shares of the chunk
prologue, token loop and flush, plus cycles per token and per chunk.

python scripts/lda_stamps.py [bench_lda args...]
"""
import ctypes
import json
import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "ab", "liblda_stamps.so")


def main():
    os.environ["HARP_KERNEL_LIB"] = LIB
    sys.argv = [os.path.join(HERE, "bench_lda.py")] + sys.argv[1:]
    try:
        runpy.run_path(sys.argv[0], run_name="__main__")
    except SystemExit:
        pass
    lib = ctypes.CDLL(LIB)
    out = (ctypes.c_ulonglong * 8)()
    assert lib.harp_lda_stamps(out, 0) == 0
    pro, tok, fl, nch, ntok, wave = [int(v) for v in out[:6]]
    tot = pro + tok + fl
    print(json.dumps({"prologue_share": pro / tot, "token_loop_share": tok / tot, "flush_share": fl / tot,
                      "chunks": nch, "tokens": ntok, "tokens_per_chunk": ntok / max(nch, 1),
                      "cycles_per_token_loop_token": tok / max(ntok, 1), "prologue_cycles_per_chunk": pro / max(nch, 1),
                      "flush_cycles_per_chunk": fl / max(nch, 1), "wave_cycles": wave, "loop_cycles": tot}))


if __name__ == "__main__":
    main()
