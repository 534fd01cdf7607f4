#!/bin/bash
# sparse sampler with wave-uniform token scalars: tests + full-size sweep; dense default variant 0
set -o pipefail
O=gpurun_out/round5_i
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lda_gpu.py tests/test_rowcodec_gpu.py tests/test_lda_pp_mp_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_lda.py --docs 1e6 --strategy push_pull --local-server off --iters 5 > $O/full_sparse.log 2>&1 || { echo full failed; tail $O/full_sparse.log; exit 1; }
tail -1 $O/full_sparse.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full sparse', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > $O/share8.log 2>&1 || { echo share failed; tail $O/share8.log; exit 1; }
tail -1 $O/share8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('share8', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
