#!/bin/bash
# MF-SGD LDS-DMA triple staging: GPU SGD tests + same-process A/B (full set, 8-GPU share)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5k
timeout -k 10 300 python -u -m pytest tests/test_sgd_mf_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5k/tests.log 2>&1 || { tail -30 gpurun_out/r5k/tests.log; exit 1; }
tail -1 gpurun_out/r5k/tests.log
timeout -k 10 200 python scripts/probe_sgd_stage.py > gpurun_out/r5k/ab_full.log 2>&1 || { tail -20 gpurun_out/r5k/ab_full.log; exit 1; }
tail -1 gpurun_out/r5k/ab_full.log
timeout -k 10 200 python scripts/probe_sgd_stage.py --ratings 12560063 --slices 16 > gpurun_out/r5k/ab_share.log 2>&1 || { tail -20 gpurun_out/r5k/ab_share.log; exit 1; }
tail -1 gpurun_out/r5k/ab_share.log
