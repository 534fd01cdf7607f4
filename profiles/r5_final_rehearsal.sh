#!/bin/bash
# final round-5 state: P = 2 one-GPU rehearsal (gloo) of the bench's LDA record, fused push-pull rows
set -o pipefail
O=gpurun_out/round5_final_rehearsal
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HARP_BENCH_TRACE=1
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 --points 2e6 --sgd off --extras on --pca-n 1e6 --pca-steps 2 --lda-docs 4e5 --lda-vocab 4e5 --lda-iters 3 --extras-timeout 300 > $O/bench_p2.log 2>&1 || { echo "bench P=2 failed"; tail -20 $O/bench_p2.log; exit 1; }
grep '^{' $O/bench_p2.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); v=r.get("lda",{}); print("P", r["n_gpus"], {a:b for a,b in v.items() if a in ("tokens_per_sec","s_per_iter","comm_mode","fused_rows","error","loglik_end","pull_ms","push_ms")})'
