#!/bin/bash
# round-3: SAHAD templates u3-1 / u5-1 / u7-1 at the Twitter graph's size (42M vertices,
# 1.2B undirected edges; BASELINE #7) on ONE MI355X: seconds per coloring
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r7o
mkdir -p $O
for K in 3 5 7; do
  timeout -k 10 400 python -u scripts/bench_subgraph.py --nodes 4.2e7 --edges 1.2e9 --k $K --iters 2 > $O/twitter_u$K.log 2>&1
  rc=$?; echo "u$K-1 rc=$rc: $(grep '^{' $O/twitter_u$K.log)"
  [ $rc -eq 0 ] || { tail -5 $O/twitter_u$K.log; exit $rc; }
done
