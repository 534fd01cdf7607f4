#!/bin/bash
# K-means partial last tile: GPU K-means tests, then bench (K = 1e4 sweeps 10,016 rows)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
timeout -k 10 300 python -u -m pytest tests/test_kmeans_gpu.py tests/test_kmeans.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d/tests.log 2>&1 || { tail -30 gpurun_out/r4d/tests.log; exit 1; }
tail -2 gpurun_out/r4d/tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --sgd off > gpurun_out/r4d/bench.log 2>&1 || { tail -20 gpurun_out/r4d/bench.log; exit 1; }
grep '^{' gpurun_out/r4d/bench.log | tail -1 | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4d/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --sgd off > $GRAFT_REPO_ROOT/gpurun_out/r4d/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4d/prof.log; exit 1; }
grep '^{' $GRAFT_REPO_ROOT/gpurun_out/r4d/prof.log | tail -1 | cut -c1-200
