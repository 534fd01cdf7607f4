#!/bin/bash
# full GPU suite + 1-GPU bench (headline + nested SGD record) after the round-2 follow-ups
set -o pipefail
mkdir -p gpurun_out/r2j
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2j/pytest.log 2>&1 || { tail -40 gpurun_out/r2j/pytest.log; exit 1; }
tail -3 gpurun_out/r2j/pytest.log
timeout -k 10 400 python bench.py > gpurun_out/r2j/bench.log 2>&1 || { tail -30 gpurun_out/r2j/bench.log; exit 1; }
tail -1 gpurun_out/r2j/bench.log
