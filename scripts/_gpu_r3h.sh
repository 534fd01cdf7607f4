#!/bin/bash
# MF-SGD full Netflix-shape: blocks_per_xcd x chunk sweep (1 GPU)
set -o pipefail
mkdir -p gpurun_out/r3h
for b in 64 128 256; do
  for c in 32 64 128; do
    timeout -k 10 120 python scripts/bench_sgd.py --epochs 5 --blocks-per-xcd $b --chunk $c > gpurun_out/r3h/b${b}_c$c.log 2>&1 || { tail -5 gpurun_out/r3h/b${b}_c$c.log; exit 1; }
    python -c "import json; r=json.loads([l for l in open('gpurun_out/r3h/b${b}_c$c.log') if l.startswith('{')][-1]); print('bpx=$b chunk=$c', round(r['s_per_epoch']*1e3,3), 'ms', round(r['train_rmse'],5))"
  done
done
