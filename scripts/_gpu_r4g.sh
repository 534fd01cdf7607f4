#!/bin/bash
# slab codec: GPU tests, LDA GPU tests, codec cost at the 8-rank LDA slab shape
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
#timeout -k 10 300 python -u -m pytest tests/test_slabcodec_gpu.py tests/test_slabcodec.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4g/tests.log 2>&1 || { tail -30 gpurun_out/r4g/tests.log; exit 1; }
#tail -1 gpurun_out/r4g/tests.log
timeout -k 10 200 python scripts/bench_slabcodec.py > gpurun_out/r4g/bench.log 2>&1 || { tail -20 gpurun_out/r4g/bench.log; exit 1; }
tail -1 gpurun_out/r4g/bench.log
timeout -k 10 200 python scripts/bench_slabcodec.py --slices 2 > gpurun_out/r4g/bench_s2.log 2>&1 || { tail -20 gpurun_out/r4g/bench_s2.log; exit 1; }
tail -1 gpurun_out/r4g/bench_s2.log
