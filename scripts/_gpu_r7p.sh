#!/bin/bash
# round-3: SAHAD templates at the NYC graph's size (18M vertices, 480M edges) on one MI355X
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r7o
mkdir -p $O
for K in 3 5 7; do
  timeout -k 10 300 python -u scripts/bench_subgraph.py --nodes 1.8e7 --edges 4.8e8 --k $K --iters 3 > $O/nyc_u$K.log 2>&1
  rc=$?; echo "nyc u$K-1 rc=$rc: $(grep '^{' $O/nyc_u$K.log | cut -c1-200)"
  [ $rc -eq 0 ] || { tail -5 $O/nyc_u$K.log; exit $rc; }
done
