#!/bin/bash
# round-3: s_setprio variants -- SYRK (1: around each stage MFMA cluster, 2: static for waves 4-7), K-means assign (15: static)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8t
mkdir -p $O
for rep in 1 2; do
  for v in 0 1 2; do
    timeout -k 10 200 python scripts/bench_pca.py --variant $v --steps 5 > $O/v${v}_$rep.log 2>&1 || { echo "v$v failed"; tail -5 $O/v${v}_$rep.log; exit 1; }
    echo "variant $v rep$rep: $(grep '^{' $O/v${v}_$rep.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["value"],5), round(r["syrk_s_local"],5), r["max_eigenvalue"])')"
  done
done
# K-means assign: variant 15 = 14 + static priority for waves 4-7
for rep in 1 2; do
  for v in 14 15; do
    timeout -k 10 200 python bench.py --variant $v --sgd off --extras off --steps 10 --warmup 2 > $O/km_v${v}_$rep.log 2>&1 || { echo "km v$v failed"; tail -5 $O/km_v${v}_$rep.log; exit 1; }
    echo "kmeans variant $v rep$rep: $(grep '^{' $O/km_v${v}_$rep.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["median_s_per_iter"], r["mean_sq_dist"])')"
  done
done
