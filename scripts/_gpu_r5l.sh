#!/bin/bash
# round-2 final app bench sweep (1 GPU): every scripts/bench_*.py at its default shape
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5l
for b in tsqr knn mds pagerank subgraph mlr kmeans_csr ccd als lda pca sgd; do
  timeout -k 10 240 python scripts/bench_$b.py > gpurun_out/r5l/$b.log 2>&1 || { echo "$b FAILED"; tail -5 gpurun_out/r5l/$b.log; exit 1; }
  echo "$b: $(grep '^{' gpurun_out/r5l/$b.log | tail -1 | cut -c1-230)"
done
