#!/bin/bash
# A/B of dense-sampler variants at the 8-GPU LDA share: each scripts/ab/<v>/libharp_kernels.so
# is copied into place and the share sweep timed (AB_FULL=1: the full size too), variants
# interleaved over two rounds
set -o pipefail
O=gpurun_out/${1:-round5_ab}
shift
mkdir -p $O
export PYTHONUNBUFFERED=1
for R in 1 2; do
  for V in "$@"; do
    cp scripts/ab/$V/libharp_kernels.so harp_amd/_native/libharp_kernels.so
    unset HARP_LDA_SOLE
    [ -f scripts/ab/$V/env ] && source scripts/ab/$V/env  # per-variant environment
    timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > $O/share8_${V}_$R.log 2>&1 || { echo share failed; tail $O/share8_${V}_$R.log; exit 1; }
    tail -1 $O/share8_${V}_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('share8 $V', d['s_per_iter'], d['loglik_end'])"
    if [ -n "$AB_FULL" ]; then
      timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --strategy push_pull --local-server off --iters 5 > $O/full_${V}_$R.log 2>&1 || { echo full failed; tail $O/full_${V}_$R.log; exit 1; }
      tail -1 $O/full_${V}_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full $V', d['s_per_iter'], d['loglik_end'])"
    fi
  done
done
