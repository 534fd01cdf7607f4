#!/bin/bash
# round-4 final check: the end-state script (GPU suite, smoke, bench, kernel stats), the LDA
# clueweb1 full share, and the sparse-LDA multi-rank rehearsal
set -o pipefail
bash profiles/r4_endstate/r4_endstate.sh || exit $?
out=gpurun_out/r4final
mkdir -p $out
timeout -k 10 420 python -u scripts/bench_lda.py --docs 9.52e6 --vocab 999933 --topics 10000 --len 392 --iters 2 \
  --warmup 1 --strategy rotation > $out/lda_k10000_full_share.log 2>&1 || exit $?
bash profiles/r4_rehearsal/r4_rehearsal_sparse.sh > $out/rehearsal_sparse.log 2>&1
