#!/bin/bash
# round-3 end-of-session app sweep: every scripts/bench_*.py at its default shape (+ LDA K = 10,000)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8l
mkdir -p $O
: > $O/summary.txt
for b in als ccd kmeans_csr knn lda mds mlr pagerank pca sgd slabcodec subgraph; do
  timeout -k 10 240 python scripts/bench_$b.py > $O/$b.log 2>&1
  rc=$?
  echo "$b rc=$rc $(grep '^{' $O/$b.log | tail -1 | cut -c1-400)" | tee -a $O/summary.txt
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 240 python scripts/bench_lda.py --topics 10000 --iters 3 > $O/lda_k1e4.log 2>&1
rc=$?; echo "lda_k1e4 rc=$rc $(grep '^{' $O/lda_k1e4.log | tail -1 | cut -c1-400)" | tee -a $O/summary.txt
exit $rc
