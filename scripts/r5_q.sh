#!/bin/bash
# dense LDA sampler, packed uint8 rows with the next token's row prefetched: tests, 8-share, full size
set -o pipefail
O=gpurun_out/round5_q
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lda_gpu.py tests/test_rowcodec_gpu.py tests/test_lda_pp_mp_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for R in 1 2; do
  timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > $O/share8_$R.log 2>&1 || { echo share failed; tail $O/share8_$R.log; exit 1; }
  tail -1 $O/share8_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('share8', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'], d.get('pull_ms'), d.get('push_ms'))"
done
HARP_LDA_SAMPLER=dense timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --strategy push_pull --local-server off --iters 5 > $O/full_dense.log 2>&1 || { echo full dense failed; tail $O/full_dense.log; exit 1; }
tail -1 $O/full_dense.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full_dense', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
