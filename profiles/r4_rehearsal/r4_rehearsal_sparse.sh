#!/bin/bash
# the full bench at P = 2 / 4 on ONE GPU (gloo + host staging) with LDA at K = 2000, so the
# push-pull record runs the sparse-doc sampler without a dense doc-topic table across ranks
export TMPDIR=/tmp
O=gpurun_out/r4rs
mkdir -p $O
for P in 2 4; do
  timeout -k 10 500 python bench.py --gpus $P --backend gloo --steps 3 --warmup 1 --points 2e7 --sgd off --extras on \
    --pca-n 1e7 --pca-steps 3 --lda-docs 2e5 --lda-vocab 2e5 --lda-topics 2000 --lda-iters 3 --extras-timeout 200 \
    > $O/bench_p$P.log 2>&1
  rc=$?; echo "bench P=$P rc=$rc"
  grep '^{' $O/bench_p$P.log | python3 -c '
import json,sys
r=json.loads(sys.stdin.read())
print("kmeans", r["value"])
for k in ("pca","lda"):
    v=r.get(k,{}); print(k, v.get("error") or {a:b for a,b in v.items() if a in ("s_per_pass","eigvec_orth_err","tokens_per_sec","n_gpus","loglik_end","comm_mode","sampler","fused_rows")})
' || tail -20 $O/bench_p$P.log
  [ $rc -eq 0 ] || exit $rc
done
