#!/bin/bash
# SYRK variant 1 (4 waves x 128x128): agreement, bottleneck split, PCA bench vs variant 0
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
timeout -k 10 120 python scripts/syrk_check.py > gpurun_out/r4b/check.log 2>&1 || { tail -20 gpurun_out/r4b/check.log; exit 1; }
tail -1 gpurun_out/r4b/check.log
timeout -k 10 300 python scripts/syrk_diag.py --modes 0,1,2,10,11,12,14 > gpurun_out/r4b/diag.log 2>&1 || { tail -20 gpurun_out/r4b/diag.log; exit 1; }
tail -1 gpurun_out/r4b/diag.log
for v in 0 1; do
  timeout -k 10 300 python scripts/bench_pca.py --variant $v > gpurun_out/r4b/pca_v$v.log 2>&1 || { tail -20 gpurun_out/r4b/pca_v$v.log; exit 1; }
  echo "v=$v $(grep '^{' gpurun_out/r4b/pca_v$v.log | tail -1 | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["syrk_s_local"],4), round(r["value"],4), r["max_eigenvalue"])')"
done
