#!/bin/bash
# Round 6: multi-rank rehearsal of the full bench on ONE GPU (gloo with host staging) --
# exercises at P > 1 the LDA owner slots (rows shared by several ranks: canonical slots
# copied per requester, pushed slots merged), the per-collective records, stats.pca with
# the chip-wide eigensolver and the eigenvector broadcast.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash scripts/gpu_rehearsal_r6.sh [outdir]'
export TMPDIR=/tmp
O=${1:-gpurun_out/r6_rehearsal}
mkdir -p $O
for P in ${PS:-2 3}; do
  HARP_BENCH_TRACE=1 timeout -k 10 500 python bench.py --gpus $P --backend gloo --steps 3 --warmup 1 --points 2e7 --sgd on --sgd-epochs 3 --extras on --pca-n 1e7 --pca-steps 3 --lda-docs 2e5 --lda-vocab 2e5 --lda-iters 3 --sgd-timeout 300 --extras-timeout 200 > $O/bench_p$P.log 2>&1
  rc=$?; echo "bench P=$P rc=$rc"
  grep '^{' $O/bench_p$P.log | tail -1 | python3 -c '
import json,sys
r=json.loads(sys.stdin.read())
print("kmeans", r["value"], r["sync_bytes_per_iter"])
for k in ("sgd","pca","lda"):
    v=r.get(k,{}); print(k, v.get("error") or {a:b for a,b in v.items() if a in ("updates_per_sec","slices_per_rank","s_per_pass","eig_s","eigvec_orth_err","tokens_per_sec","n_gpus","max_eigenvalue","train_rmse","loglik_end","comm_mode","fused_rows")})
' || tail -20 $O/bench_p$P.log
  [ $rc -eq 0 ] || exit $rc
done
