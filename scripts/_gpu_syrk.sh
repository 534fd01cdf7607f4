#!/bin/bash
# SYRK co-residency sweep at N=1e8 x d=1000: 24 splits = 240 co-resident workgroups (3 splits x 10 tiles per XCD)
set -o pipefail
mkdir -p gpurun_out/syrk2
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/syrk2/pytest.log 2>&1 || { tail -30 gpurun_out/syrk2/pytest.log; exit 1; }
tail -2 gpurun_out/syrk2/pytest.log
for cfg in "0 24" "4 24" "3 24" "4 0" "0 48" "4 48" "4 16"; do set -- $cfg
  timeout -k 10 300 python scripts/bench_pca.py --variant $1 --splits $2 --steps 2 > gpurun_out/syrk2/v$1_s$2.log 2>&1 || { tail -20 gpurun_out/syrk2/v$1_s$2.log; exit 1; }
  echo "v$1 s$2 $(grep -o '"syrk_s_local": [0-9.e-]*' gpurun_out/syrk2/v$1_s$2.log)"
done
