#!/bin/bash
# MF-SGD rank 2000: does an L2-sized H block per XCD change the update rate? items 17770 vs 2222 vs 1111
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4o
for it in 17770 2222 1111; do
  timeout -k 10 200 python scripts/bench_sgd.py --rank 2000 --items $it --ratings 20000000 --chunk 0 --epochs 3 --warmup 1 > gpurun_out/r4o/items$it.log 2>&1 || { tail -20 gpurun_out/r4o/items$it.log; exit 1; }
  echo "items=$it $(grep '^{' gpurun_out/r4o/items$it.log | tail -1 | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", "%.3e" % r["value"], "upd/s")')"
done
