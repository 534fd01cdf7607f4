#!/bin/bash
# new-kernel GPU tests (TSQR, NN epilogues, SGD budget), then the full gpu suite
set -o pipefail
mkdir -p gpurun_out/r2d
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py tests/test_nn_gpu.py tests/test_sgd_mf_gpu.py tests/test_kmeans_csr_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2d/new.log 2>&1 || { tail -40 gpurun_out/r2d/new.log; exit 1; }
tail -2 gpurun_out/r2d/new.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2d/pytest.log 2>&1 || { tail -40 gpurun_out/r2d/pytest.log; exit 1; }
tail -2 gpurun_out/r2d/pytest.log
