#!/bin/bash
# LDA one-lane doc-row atomics at uniform base + VGPR byte offset: tests, full-size P=1 push-pull and 8-share, twice
set -o pipefail
O=gpurun_out/${1:-round5_oo}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lda_gpu.py tests/test_rowcodec_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for R in 1 2; do
  timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --strategy push_pull --local-server off --iters 5 > $O/full_$R.log 2>&1 || { echo full failed; tail $O/full_$R.log; exit 1; }
  tail -1 $O/full_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
  timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > $O/share8_$R.log 2>&1 || { echo share failed; tail $O/share8_$R.log; exit 1; }
  tail -1 $O/share8_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('share8', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
done
