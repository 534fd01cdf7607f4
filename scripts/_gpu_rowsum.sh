#!/bin/bash
# gather-sum unroll 4 vs 8: kernel-trace stats of a short bench
set -o pipefail
mkdir -p gpurun_out/rowsum
cd /tmp && export TMPDIR=/tmp
for u in 4 8; do
  HARP_ROWSUM_UNROLL=$u timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/rowsum/u$u -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --sgd off > $GRAFT_REPO_ROOT/gpurun_out/rowsum/u$u.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/rowsum/u$u.log; exit 1; }
  echo "u$u $(tail -1 $GRAFT_REPO_ROOT/gpurun_out/rowsum/u$u.log | grep -o '"value": [0-9.]*')"
done
