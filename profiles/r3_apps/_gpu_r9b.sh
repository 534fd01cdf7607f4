#!/bin/bash
# round-3: scripts/bench_pca.py (one-XCD eig, upper-triangle FLOP/s) and bench_sgd.py (one slice) at defaults
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r9b
mkdir -p $O
for b in pca sgd; do
  timeout -k 10 240 python scripts/bench_$b.py > $O/$b.log 2>&1
  rc=$?; echo "$b rc=$rc $(grep '^{' $O/$b.log | tail -1 | cut -c1-330)"
  [ $rc -eq 0 ] || exit $rc
done
