#!/bin/bash
# round-3: MF-SGD flow kernel (one launch per slice pass, cross-XCD completion flags) at FULL size
# with one slice per rank and hot-weighted blocks, vs per-sub-step launches (alternating)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r9g
mkdir -p $O
for rep in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python scripts/bench_sgd.py --epochs 10 --variant $v > $O/full_v${v}_$rep.log 2>&1 || { tail -5 $O/full_v${v}_$rep.log; exit 1; }
    echo "rep $rep variant $v: $(grep '^{' $O/full_v${v}_$rep.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", round(r["train_rmse"],5))')"
  done
done
