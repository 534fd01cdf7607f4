#!/bin/bash
# MF-SGD rank-share rehearsal on 1 GPU: slice-steps per epoch = P x S for S = 2 (default) vs S = 1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
for cfg in "12560063 16" "12560063 8" "25120127 8" "25120127 4" "50240254 4" "50240254 2"; do
  set -- $cfg
  timeout -k 10 180 python bench.py --points 1e6 --steps 2 --warmup 1 --sgd on --sgd-ratings $1 --sgd-slices $2 --sgd-epochs 10 --sgd-warmup 2 > gpurun_out/r4f/r$1_s$2.log 2>&1 || { tail -20 gpurun_out/r4f/r$1_s$2.log; exit 1; }
  echo "ratings=$1 slices=$2 $(grep '^{' gpurun_out/r4f/r$1_s$2.log | tail -1 | python -c 'import json,sys; r=json.loads(sys.stdin.read())["sgd"]; print(round(r["s_per_epoch"]*1e3,3), "ms", r["updates_per_sec"], r["train_rmse"])')"
done
