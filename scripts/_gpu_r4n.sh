#!/bin/bash
# MF-SGD 8-GPU rank share (12.56M ratings, 16 slice steps): blocks_per_xcd x chunk sweep
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4n
for b in 64 128 256 512; do
  for c in 8 16; do
    timeout -k 10 120 python scripts/bench_sgd.py --ratings 12560063 --slices 16 --chunk $c --blocks-per-xcd $b --epochs 10 --warmup 2 > gpurun_out/r4n/b${b}_c$c.log 2>&1 || { tail -20 gpurun_out/r4n/b${b}_c$c.log; exit 1; }
    echo "bpx=$b chunk=$c $(grep '^{' gpurun_out/r4n/b${b}_c$c.log | tail -1 | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", round(r["train_rmse"],6))')"
  done
done
