#!/bin/bash
# dense LDA sampler: five (variant 0) vs six (variant 3) waves per SIMD at the 8-GPU share and full size
set -o pipefail
O=gpurun_out/round5_n
mkdir -p $O
export PYTHONUNBUFFERED=1
for V in 0 3 0 3; do
  HARP_LDA_VARIANT=$V timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > $O/share8_v$V.log 2>&1 || { echo share failed; tail $O/share8_v$V.log; exit 1; }
  tail -1 $O/share8_v$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('share8 v$V', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
done
for V in 0 3; do
  HARP_LDA_VARIANT=$V HARP_LDA_SAMPLER=dense timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --strategy push_pull --local-server off --iters 5 > $O/full_dense_v$V.log 2>&1 || { echo full failed; tail $O/full_dense_v$V.log; exit 1; }
  tail -1 $O/full_dense_v$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full_dense v$V', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
done
