#!/bin/bash
# round 5: the P=4 one-GPU rehearsal (gloo, host staging) with per-rank setup traces
export TMPDIR=/tmp HARP_BENCH_TRACE=1
O=gpurun_out/round5_y
mkdir -p $O
( while sleep 30; do date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 600 python bench.py --gpus 4 --backend gloo --steps 3 --warmup 1 --points 2e7 --sgd on --sgd-epochs 3 --extras on --pca-n 1e7 --pca-steps 3 --lda-docs 2e5 --lda-vocab 2e5 --lda-iters 3 --sgd-timeout 300 --extras-timeout 200 > $O/bench_p4.log 2>&1
rc=$?
kill $HB
echo "bench P=4 rc=$rc"
grep "bench trace\|bench:" $O/bench_p4.log | tail -30
exit $rc
