#!/bin/bash
# round-3: the r8o 3-rank rehearsal command with setup tracing (LDA setup took 31 s there)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8s
mkdir -p $O
HARP_BENCH_TRACE=1 timeout -k 10 420 python -u bench.py --gpus 3 --backend gloo --steps 3 --warmup 1 --points 2e7 --sgd on --sgd-epochs 3 --extras on --pca-n 1e7 --pca-steps 3 --lda-docs 2e5 --lda-vocab 2e5 --lda-iters 3 --sgd-timeout 300 --extras-timeout 200 > $O/bench_p3.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 20; echo "hb: $(grep -c 'bench trace' $O/bench_p3.log) trace lines"; done
wait $pid; rc=$?; echo "rc=$rc"; grep "bench trace rank 0" $O/bench_p3.log
