#!/bin/bash
# SYRK with the 64-sample-blocked feature-major layout: numerics, bottleneck split, PCA bench
set -o pipefail
mkdir -p gpurun_out/syrk8
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/syrk8/pytest.log 2>&1 || { tail -30 gpurun_out/syrk8/pytest.log; exit 1; }
tail -1 gpurun_out/syrk8/pytest.log
timeout -k 10 300 python scripts/syrk_diag.py > gpurun_out/syrk8/diag.log 2>&1 || { tail -20 gpurun_out/syrk8/diag.log; exit 1; }
tail -1 gpurun_out/syrk8/diag.log
for s in 0 32; do
  HARP_SYRK_SYNC=$s timeout -k 10 300 python scripts/bench_pca.py > gpurun_out/syrk8/pca_sync$s.log 2>&1 || { tail -20 gpurun_out/syrk8/pca_sync$s.log; exit 1; }
  echo "sync=$s $(grep '^{' gpurun_out/syrk8/pca_sync$s.log | tail -1)"
done
