#!/bin/bash
# SYRK lock-step interval sweep + L2 hit counters with / without the lock-step
set -o pipefail
mkdir -p gpurun_out/syrk4
for sy in 16 24 48 64; do
  HARP_SYRK_SYNC=$sy timeout -k 10 300 python scripts/bench_pca.py --steps 2 > gpurun_out/syrk4/sync$sy.log 2>&1 || { tail -20 gpurun_out/syrk4/sync$sy.log; exit 1; }
  echo "sync$sy $(grep -o '"syrk_s_local": [0-9.e-]*' gpurun_out/syrk4/sync$sy.log)"
done
cd /tmp && export TMPDIR=/tmp
for sy in 0 32; do
  HARP_SYRK_SYNC=$sy timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_BUSY_CYCLES -d $GRAFT_REPO_ROOT/gpurun_out/syrk4/pmc$sy -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_pca.py --n 2e7 --steps 1 --warmup 0 > $GRAFT_REPO_ROOT/gpurun_out/syrk4/pmc$sy.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/syrk4/pmc$sy.log; exit 1; }
  echo "pmc$sy done"
done
