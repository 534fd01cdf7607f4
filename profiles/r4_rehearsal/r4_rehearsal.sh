#!/bin/bash
# round 4: multi-rank rehearsal of the full bench on ONE GPU (gloo with host staging):
# exercises at P > 1 the new code paths -- two MF-SGD slices per rank, stats.pca with the
# eigenvector broadcast, fused LDA push-pull rows, header-free ring rotation
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
for P in 2 4; do
  timeout -k 10 500 python bench.py --gpus $P --backend gloo --steps 3 --warmup 1 --points 2e7 --sgd on --sgd-epochs 3 --extras on --pca-n 1e7 --pca-steps 3 --lda-docs 2e5 --lda-vocab 2e5 --lda-iters 3 --sgd-timeout 300 --extras-timeout 200 > $O/bench_p$P.log 2>&1
  rc=$?; echo "bench P=$P rc=$rc"
  grep '^{' $O/bench_p$P.log | python3 -c '
import json,sys
r=json.loads(sys.stdin.read())
print("kmeans", r["value"], r["sync_bytes_per_iter"])
for k in ("sgd","pca","lda"):
    v=r.get(k,{}); print(k, v.get("error") or {a:b for a,b in v.items() if a in ("updates_per_sec","slices_per_rank","s_per_pass","eig_s","eigvec_orth_err","tokens_per_sec","sync_bytes_per_iter","n_gpus","max_eigenvalue","train_rmse","loglik_end","comm_mode","fused_rows")})
' || tail -20 $O/bench_p$P.log
  [ $rc -eq 0 ] || exit $rc
done
