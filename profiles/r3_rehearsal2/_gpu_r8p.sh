#!/bin/bash
# round-3: 4-rank rehearsal of the full bench on ONE GPU (gloo + host staging), with a
# heartbeat so a slow (not hung) run is not taken for silent
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8p
mkdir -p $O
P=4
timeout -k 10 900 python -u bench.py --gpus $P --backend gloo --steps 3 --warmup 1 --points 2e7 --sgd on --sgd-epochs 3 --extras on --pca-n 1e7 --pca-steps 3 --lda-docs 2e5 --lda-vocab 2e5 --lda-iters 3 --sgd-timeout 400 --extras-timeout 300 > $O/bench_p$P.log 2>&1 &
pid=$!
t=0
while kill -0 $pid 2>/dev/null; do sleep 30; t=$((t+30)); echo "heartbeat ${t}s: $(grep -c . $O/bench_p$P.log) log lines"; done
wait $pid; rc=$?
echo "bench P=$P rc=$rc"
grep '^{' $O/bench_p$P.log | python3 -c '
import json,sys
r=json.loads(sys.stdin.read())
print("kmeans", r["value"], r["sync_bytes_per_iter"])
for k in ("sgd","pca","lda"):
    v=r.get(k,{}); print(k, v.get("error") or {a:b for a,b in v.items() if a in ("updates_per_sec","s_per_pass","tokens_per_sec","sync_bytes_per_iter","n_gpus","max_eigenvalue","train_rmse","loglik_end","setup_s")})
' || tail -20 $O/bench_p$P.log
exit $rc
