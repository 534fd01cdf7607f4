#!/bin/bash
# multi-stage SYRK ring without the __syncthreads vmcnt drain, with / without the split lock-step
set -o pipefail
mkdir -p gpurun_out/syrk5
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/syrk5/pytest.log 2>&1 || { tail -30 gpurun_out/syrk5/pytest.log; exit 1; }
tail -1 gpurun_out/syrk5/pytest.log
for cfg in "1 0" "1 32" "1 64" "1 128" "0 32"; do set -- $cfg
  HARP_SYRK_SYNC=$2 timeout -k 10 300 python scripts/bench_pca.py --variant $1 --steps 2 > gpurun_out/syrk5/v$1_sync$2.log 2>&1 || { tail -20 gpurun_out/syrk5/v$1_sync$2.log; exit 1; }
  echo "v$1 sync$2 $(grep -o '"syrk_s_local": [0-9.e-]*' gpurun_out/syrk5/v$1_sync$2.log) $(grep -o '"max_eigenvalue": [0-9.e-]*' gpurun_out/syrk5/v$1_sync$2.log)"
done
