#!/bin/bash
# LDA-CGS at the clueweb1 shape (K = 10,000, 999,933 words, 392 tokens per document):
# GPU tests of the no-dense-doc-table sparse path, then one 8-GPU rank's half and full
# share (4.76M / 9.52M documents, 1.87e9 / 3.73e9 tokens) on one MI355X
# (profiles/r4_published/README.md).
set -o pipefail
out=gpurun_out/r4lda_cw
mkdir -p $out
(while sleep 45; do date +%T >> $out/heartbeat.txt; done) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lda_gpu.py \
  tests/test_rowcodec_gpu.py tests/test_lda_pp_mp_gpu.py > $out/pytest.log 2>&1 || exit $?
for docs in 4.76e6 9.52e6; do
  timeout -k 10 420 python -u scripts/bench_lda.py --docs $docs --vocab 999933 --topics 10000 --len 392 --iters 2 \
    --warmup 1 --strategy rotation > $out/lda_k10000_docs$docs.log 2>&1
  rc=$?; echo "docs $docs rc=$rc" >> $out/status.txt; [ $rc -eq 0 ] || exit $rc
done
