#!/bin/bash
# round-3: hot-row weighted item blocks, repeat A/B at the default skew (full size and 8-GPU share)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r9e
mkdir -p $O
for rep in 1 2; do
  for h in 0 1 0.75; do
    HARP_SGD_HOT=$h timeout -k 10 200 python scripts/bench_sgd.py --epochs 10 > $O/full_h${h}_$rep.log 2>&1 || exit 1
    HARP_SGD_HOT=$h timeout -k 10 200 python scripts/bench_sgd.py --epochs 10 --users 60024 --ratings 12560064 --slices 8 > $O/s8_h${h}_$rep.log 2>&1 || exit 1
    echo "rep $rep hot $h: full $(grep '^{' $O/full_h${h}_$rep.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", round(r["train_rmse"],5))') | share8 $(grep '^{' $O/s8_h${h}_$rep.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", round(r["train_rmse"],5))')"
  done
done
