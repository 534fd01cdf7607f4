#!/bin/bash
# ALS wave-per-system Cholesky: GPU ALS tests, kernel split probe, ALS bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5h
timeout -k 10 300 python -u -m pytest tests/test_als_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5h/tests.log 2>&1 || { tail -30 gpurun_out/r5h/tests.log; exit 1; }
tail -1 gpurun_out/r5h/tests.log
timeout -k 10 300 python scripts/bench_als.py > gpurun_out/r5h/bench_als.log 2>&1 || { tail -20 gpurun_out/r5h/bench_als.log; exit 1; }
tail -1 gpurun_out/r5h/bench_als.log | cut -c1-300
timeout -k 10 200 python scripts/probe_als.py > gpurun_out/r5h/probe.log 2>&1 || { tail -20 gpurun_out/r5h/probe.log; exit 1; }; tail -1 gpurun_out/r5h/probe.log
