#!/bin/bash
# round-3: trace of the LDA record's setup in the 3-rank one-GPU rehearsal (gloo + staging)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8r
mkdir -p $O
HARP_BENCH_TRACE=1 timeout -k 10 400 python -u bench.py --gpus 3 --backend gloo --steps 2 --warmup 1 --points 2e6 --sgd on --sgd-epochs 2 --extras on --pca-n 1e6 --pca-steps 2 --lda-docs 2e5 --lda-vocab 2e5 --lda-iters 2 --extras-timeout 300 --sgd-timeout 300 > $O/bench_p3.log 2>&1
rc=$?; echo "rc=$rc"; grep "bench trace" $O/bench_p3.log; grep '^{' $O/bench_p3.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["lda"].get("setup_s"), r["lda"].get("error"))'
