#!/bin/bash
# dense LDA sampler, inverse topic sums from global memory (20.5 KB LDS per workgroup): six (variant 0) vs seven (3) waves per SIMD
set -o pipefail
O=gpurun_out/round5_ee
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lda_gpu.py tests/test_rowcodec_gpu.py tests/test_lda_pp_mp_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for V in 0 3 0 3; do
  HARP_LDA_VARIANT=$V timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > $O/share8_v$V.log 2>&1 || { echo share failed; tail $O/share8_v$V.log; exit 1; }
  tail -1 $O/share8_v$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('share8 v$V', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
done
for V in 0 3; do
  HARP_LDA_VARIANT=$V timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --strategy push_pull --local-server off --iters 5 > $O/full_v$V.log 2>&1 || { echo full failed; tail $O/full_v$V.log; exit 1; }
  tail -1 $O/full_v$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full v$V', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
done
