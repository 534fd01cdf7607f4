#!/bin/bash
# dense LDA sampler: one-lane token updates by dynamic register indexing (no if-converted
# selects over all 16 topic registers); tests + 8-share sweep at both occupancy variants
set -o pipefail
O=gpurun_out/round5_h
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lda_gpu.py tests/test_rowcodec_gpu.py tests/test_lda_pp_mp_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for V in 0 3; do
  HARP_LDA_VARIANT=$V timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > $O/share8_v$V.log 2>&1 || { echo share failed; tail $O/share8_v$V.log; exit 1; }
  tail -1 $O/share8_v$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant', $V, d['s_per_iter'], d['value'], d['loglik_end'])"
done
HARP_LDA_SAMPLER=dense HARP_LDA_VARIANT=0 timeout -k 10 300 python -u scripts/bench_lda.py --docs 1e6 --strategy push_pull --local-server off --iters 5 > $O/full_dense_v0.log 2>&1 || { echo full failed; tail $O/full_dense_v0.log; exit 1; }
tail -1 $O/full_dense_v0.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full dense v0', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
timeout -k 10 300 python -u scripts/bench_lda.py --docs 1e6 --strategy push_pull --local-server off --iters 5 > $O/full_sparse.log 2>&1 || { echo full failed; tail $O/full_sparse.log; exit 1; }
tail -1 $O/full_sparse.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('full sparse', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
