#!/bin/bash
# One 8-GPU rank's share of the reference's published clueweb runs (BASELINE rows 1-6), on
# one MI355X: MF-SGD rank 2000 and MF-CCD rank 120 on the clueweb2 shape (76,163,963 x
# 999,933; a rank holds 1/8 of the users), LDA-CGS K = 10,000 on the clueweb1 shape
# (999,933 words, 392 tokens per document). Ratings / tokens are a sample of the share; the
# per-update / per-token rates carry over (profiles/r4_published/README.md).
set -o pipefail
out=gpurun_out/r4pub
mkdir -p $out
# progress marker for the box's idle detector (every step below has its own time limit)
(while sleep 45; do date +%T >> $out/heartbeat.txt; done) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 420 python -u scripts/bench_sgd.py --users 9520495 --items 999933 --ratings 400000000 --rank 2000 \
  --epochs 2 --warmup 1 --lr 0.001 --lam 0.01 > $out/sgd_r2000.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_ccd.py --users 9520495 --items 999933 --ratings 4e8 --rank 120 \
  --iters 2 > $out/ccd_r120.log 2>&1 &&
timeout -k 10 360 python -u scripts/bench_lda.py --docs 1e6 --vocab 999933 --topics 10000 --len 392 --iters 2 \
  --warmup 1 --strategy rotation > $out/lda_k10000.log 2>&1
rc=$?
echo "rc=$rc" >> $out/status.txt
exit $rc
