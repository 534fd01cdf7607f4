#!/bin/bash
# round-3 (one-slice SGD default): 2-, 3- and 4-rank rehearsal of the full bench (every nested record) on ONE GPU:
# gloo transport with host staging (RCCL refuses two ranks per device), all kernels on the GPU
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8o
mkdir -p $O
for P in 2 3 4; do
  timeout -k 10 420 python bench.py --gpus $P --backend gloo --steps 3 --warmup 1 --points 2e7 --sgd on --sgd-epochs 3 --extras on --pca-n 1e7 --pca-steps 3 --lda-docs 2e5 --lda-vocab 2e5 --lda-iters 3 --sgd-timeout 300 --extras-timeout 200 > $O/bench_p$P.log 2>&1
  rc=$?; echo "bench P=$P rc=$rc"
  grep '^{' $O/bench_p$P.log | python3 -c '
import json,sys
r=json.loads(sys.stdin.read())
print("kmeans", r["value"], r["sync_bytes_per_iter"])
for k in ("sgd","pca","lda"):
    v=r.get(k,{}); print(k, v.get("error") or {a:b for a,b in v.items() if a in ("updates_per_sec","s_per_pass","tokens_per_sec","sync_bytes_per_iter","n_gpus","max_eigenvalue","train_rmse","loglik_end")})
' || tail -20 $O/bench_p$P.log
  [ $rc -eq 0 ] || exit $rc
done
