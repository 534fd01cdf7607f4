#!/bin/bash
# one 8-GPU rank's full share of the reference's clueweb1 LDA run (K = 10,000, 9.52M docs x 392 tokens =
# 3.73e9 tokens) on one MI355X with the round-5 sparse sampler (token ids two ahead, one word slice per worker)
set -o pipefail
O=gpurun_out/round5_ll
mkdir -p $O
(while sleep 45; do date +%T >> $O/heartbeat.txt; done) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u scripts/bench_lda.py --docs 9.52e6 --vocab 999933 --topics 10000 --len 392 --iters 2 \
  --warmup 1 --strategy rotation > $O/lda_k10000_full_share.log 2>&1
rc=$?
tail -1 $O/lda_k10000_full_share.log | cut -c1-600
exit $rc
