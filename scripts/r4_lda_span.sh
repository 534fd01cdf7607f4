#!/bin/bash
# sparse LDA sampler: per-token doc spans (HARP_LDA_SPAN=1) vs doc ids -> doc_off (0)
set -o pipefail
out=gpurun_out/r4span
mkdir -p $out
(while sleep 45; do date +%T >> $out/heartbeat.txt; done) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lda_gpu.py tests/test_rowcodec_gpu.py > $out/pytest.log 2>&1 || exit $?
for r in 1 2; do
  for sp in 1 0; do
    HARP_LDA_SPAN=$sp timeout -k 10 300 python -u scripts/bench_lda.py --iters 5 > $out/cfg5_rot_span${sp}_$r.log 2>&1 || exit $?
    HARP_LDA_SPAN=$sp timeout -k 10 300 python -u scripts/bench_lda.py --docs 4.76e6 --vocab 999933 --topics 10000 --len 392 \
      --iters 2 --warmup 1 > $out/cw_half_span${sp}_$r.log 2>&1 || exit $?
  done
done
