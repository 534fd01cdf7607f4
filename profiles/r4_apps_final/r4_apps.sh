#!/bin/bash
# round-4 app sweep: every scripts/bench_*.py at its default shape, plus the speed gates
mkdir -p gpurun_out/r4apps
export TMPDIR=/tmp
for b in als ccd kmeans_csr knn lda mds mlr pagerank pca sgd subgraph slabcodec tsqr kmeans_wide; do
  timeout -k 10 300 python -u scripts/bench_$b.py > gpurun_out/r4apps/$b.log 2>&1
  rc=$?; echo "$b rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
timeout -k 10 300 python -u scripts/bench_lda.py --topics 10000 > gpurun_out/r4apps/lda_k1e4.log 2>&1; echo "lda_k1e4 rc=$?"
timeout -k 10 600 python -u scripts/bench_speedups.py > gpurun_out/r4apps/speedups.log 2>&1; echo "speedups rc=$?"
