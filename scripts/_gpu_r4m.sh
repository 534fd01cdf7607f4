#!/bin/bash
# MF-SGD XCD kernel: non-temporal W stores (variant 1) vs default, 8-GPU share and full set
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4m
for cfg in "12560063 16" "100480507 2"; do
  set -- $cfg
  for v in 0 1 0 1; do
    timeout -k 10 120 python scripts/bench_sgd.py --ratings $1 --slices $2 --chunk 0 --epochs 10 --warmup 2 --variant $v > gpurun_out/r4m/r$1_v$v.log 2>&1 || { tail -20 gpurun_out/r4m/r$1_v$v.log; exit 1; }
    echo "ratings=$1 slices=$2 v=$v $(grep '^{' gpurun_out/r4m/r$1_v$v.log | tail -1 | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", round(r["train_rmse"],6))')"
  done
done
