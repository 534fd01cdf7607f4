#!/bin/bash
# round-2 re-entry validation of the committed tree: GPU suite, smoke, 1-GPU bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4h/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r4h/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r4h/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4h/smoke.log 2>&1 || { tail -20 gpurun_out/r4h/smoke.log; exit 1; }
tail -1 gpurun_out/r4h/smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r4h/bench.log 2>&1 || { tail -20 gpurun_out/r4h/bench.log; exit 1; }
grep '^{' gpurun_out/r4h/bench.log | tail -1
