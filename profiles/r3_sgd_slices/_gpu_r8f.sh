#!/bin/bash
# round-3: MF-SGD launch geometry at one slice per rank (full Netflix shape; 8-GPU share)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8f
mkdir -p $O
for B in 64 128 256; do
  for C in 64 128; do
    timeout -k 10 200 python scripts/bench_sgd.py --slices 1 --epochs 10 --chunk $C --blocks-per-xcd $B > $O/full_b${B}_c$C.log 2>&1 || { echo "full B$B C$C failed"; tail -5 $O/full_b${B}_c$C.log; exit 1; }
    echo "full B=$B C=$C: $(grep '^{' $O/full_b${B}_c$C.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", r["train_rmse"])')"
  done
done
for B in 64 128 256; do
  for C in 0 16 32; do
    timeout -k 10 200 python scripts/bench_sgd.py --users 60024 --ratings 12560064 --slices 8 --epochs 10 --chunk $C --blocks-per-xcd $B > $O/s8_b${B}_c$C.log 2>&1 || { echo "s8 B$B C$C failed"; tail -5 $O/s8_b${B}_c$C.log; exit 1; }
    echo "share8 B=$B C=$C: $(grep '^{' $O/s8_b${B}_c$C.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", r["train_rmse"])')"
  done
done
