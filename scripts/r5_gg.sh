#!/bin/bash
# LDA defaults after the sampler-choice change: tests, full-size P=1 push-pull (auto -> dense), 8-share at max chunk 2048 vs auto (4069)
set -o pipefail
O=gpurun_out/round5_gg
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lda_gpu.py tests/test_rowcodec_gpu.py tests/test_lda_pp_mp_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for R in 1 2; do
  timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --strategy push_pull --local-server off --iters 5 > $O/full_$R.log 2>&1 || { echo full failed; tail $O/full_$R.log; exit 1; }
  tail -1 $O/full_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full auto', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
  for MC in 2048 0; do
    timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 --max-chunk $MC > $O/share8_mc${MC}_$R.log 2>&1 || { echo share failed; tail $O/share8_mc${MC}_$R.log; exit 1; }
    tail -1 $O/share8_mc${MC}_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('share8 mc=$MC', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
  done
done
