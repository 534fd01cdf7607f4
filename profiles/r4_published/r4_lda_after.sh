#!/bin/bash
# LDA after the sparse-sampler load batching: the clueweb1 full share (K = 10,000) and the
# bench's config #5 shape (1M docs x 1M words x 1000 topics, push-pull) (profiles/r4_published)
set -o pipefail
out=gpurun_out/r4ldaafter
mkdir -p $out
(while sleep 45; do date +%T >> $out/heartbeat.txt; done) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 420 python -u scripts/bench_lda.py --docs 9.52e6 --vocab 999933 --topics 10000 --len 392 --iters 2 \
  --warmup 1 --strategy rotation > $out/lda_k10000_full_share.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/bench_lda.py --docs 1e6 --vocab 1e6 --topics 1000 --len 100 --iters 5 \
  --warmup 1 --strategy push_pull > $out/lda_config5.log 2>&1
