#!/bin/bash
# full-size P=1 push-pull: dense sampler at max chunk 2048 / 8192 / 32768 vs the sparse sampler (speed and likelihood)
set -o pipefail
O=gpurun_out/round5_t
mkdir -p $O
export PYTHONUNBUFFERED=1
for MC in 2048 8192 32768; do
  HARP_LDA_SAMPLER=dense timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --strategy push_pull --local-server off --iters 5 --max-chunk $MC > $O/dense_$MC.log 2>&1 || { echo dense failed; tail $O/dense_$MC.log; exit 1; }
  tail -1 $O/dense_$MC.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dense mc=$MC', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
done
timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --strategy push_pull --local-server off --iters 5 > $O/sparse.log 2>&1 || { echo sparse failed; tail $O/sparse.log; exit 1; }
tail -1 $O/sparse.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sparse', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
