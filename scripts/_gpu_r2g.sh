#!/bin/bash
# LDA push-pull with sparse push / pull (1 GPU) + lda gpu tests
set -o pipefail
mkdir -p gpurun_out/r2g
timeout -k 10 300 python -u -m pytest tests/test_lda_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2g/pytest.log 2>&1 || { tail -30 gpurun_out/r2g/pytest.log; exit 1; }
tail -1 gpurun_out/r2g/pytest.log
timeout -k 10 300 python scripts/bench_lda.py --strategy push_pull > gpurun_out/r2g/lda_pp.log 2>&1 || { tail -20 gpurun_out/r2g/lda_pp.log; exit 1; }
tail -1 gpurun_out/r2g/lda_pp.log | cut -c1-250
timeout -k 10 300 python scripts/bench_lda.py --strategy push_pull --topics 10000 > gpurun_out/r2g/lda_pp_k1e4.log 2>&1 || { tail -20 gpurun_out/r2g/lda_pp_k1e4.log; exit 1; }
tail -1 gpurun_out/r2g/lda_pp_k1e4.log | cut -c1-250
