#!/bin/bash
# round-3: MF-SGD full Netflix shape on one GPU, 1 vs 2 H slices per rank; bench record with --sgd-slices 1
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8e
mkdir -p $O
for S in 1 2; do
  timeout -k 10 200 python scripts/bench_sgd.py --slices $S --epochs 10 --chunk 0 > $O/full_s$S.log 2>&1 || { echo "full S$S failed"; tail -5 $O/full_s$S.log; exit 1; }
  echo "P=1 S=$S: $(grep '^{' $O/full_s$S.log | cut -c1-240)"
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --extras off --sgd-slices 1 > $O/bench_s1.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_s1.log; exit 1; }
grep '^{' $O/bench_s1.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print({k: v for k, v in r["sgd"].items() if not isinstance(v, (dict, list))})'
