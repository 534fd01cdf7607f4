#!/bin/bash
# round-3: every bench record at ONE RANK'S SHARE of the 2/4/8-GPU runs, on one GPU (what each
# rank computes; the collectives are not in it): K-means N/P, SGD the rank's users/ratings with
# P slices, PCA N/P, LDA docs/P over the full vocabulary
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8v
mkdir -p $O
for P in 2 4 8; do
  U=$(( (480189 + P - 1) / P )); R=$(( (100480507 + P - 1) / P ))
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --points $((100000000 / P)) --sgd-users $U --sgd-ratings $R --sgd-slices $P --pca-n $((100000000 / P)) --lda-docs $((1000000 / P)) > $O/share$P.log 2>&1
  rc=$?; echo "P=$P rc=$rc"
  grep '^{' $O/share$P.log | python3 -c '
import json,sys
r=json.loads(sys.stdin.read())
print("  kmeans", r["value"], "| sgd s/epoch", r["sgd"].get("s_per_epoch"), "| pca s/pass", r["pca"].get("s_per_pass"), "syrk", r["pca"].get("syrk_s"), "| lda s/iter", r["lda"].get("s_per_iter"), "no-local", r["lda"].get("no_local_server", {}).get("s_per_iter"))'
  [ $rc -eq 0 ] || exit $rc
done
