#!/bin/bash
# SYRK split lock-step sweep (HARP_SYRK_SYNC = stages between sync points; 0 = off)
set -o pipefail
mkdir -p gpurun_out/syrk3
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/syrk3/pytest.log 2>&1 || { tail -30 gpurun_out/syrk3/pytest.log; exit 1; }
tail -1 gpurun_out/syrk3/pytest.log
for sy in 0 8 32 128; do
  HARP_SYRK_SYNC=$sy timeout -k 10 300 python scripts/bench_pca.py --steps 2 > gpurun_out/syrk3/sync$sy.log 2>&1 || { tail -20 gpurun_out/syrk3/sync$sy.log; exit 1; }
  echo "sync$sy $(grep -o '"syrk_s_local": [0-9.e-]*' gpurun_out/syrk3/sync$sy.log) $(grep -o '"max_eigenvalue": [0-9.e-]*' gpurun_out/syrk3/sync$sy.log)"
done
