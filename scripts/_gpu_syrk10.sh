#!/bin/bash
# SYRK ring: lock-step interval sweep
set -o pipefail
mkdir -p gpurun_out/syrk10
for s in 0 32 64; do
  HARP_SYRK_SYNC=$s timeout -k 10 300 python scripts/bench_pca.py > gpurun_out/syrk10/pca_sync$s.log 2>&1 || { tail -20 gpurun_out/syrk10/pca_sync$s.log; exit 1; }
  echo "sync=$s $(grep '^{' gpurun_out/syrk10/pca_sync$s.log | tail -1 | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["syrk_s_local"],4), round(r["value"],4), r["max_eigenvalue"])')"
done
