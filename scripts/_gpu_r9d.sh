#!/bin/bash
# round-3: MF-SGD item blocks balanced by a hot-row cost weight (HARP_SGD_HOT), skew 2 and 3
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r9d
mkdir -p $O
for sk in 2.0 3.0; do
  for h in 0 0.5 1 2 4; do
    HARP_SGD_HOT=$h timeout -k 10 200 python scripts/bench_sgd.py --epochs 10 --skew $sk > $O/sk${sk}_h$h.log 2>&1 || exit 1
    echo "skew $sk hot $h: $(grep '^{' $O/sk${sk}_h$h.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", round(r["train_rmse"],5))')"
  done
done
