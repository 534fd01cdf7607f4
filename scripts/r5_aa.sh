#!/bin/bash
# sparse LDA sampler without lane branches in the register-list paths: A/B determinism, tests, K = 10,000 rotation, K = 1000 sparse full size
set -o pipefail
O=gpurun_out/round5_aa
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/lda_ab_det.py scripts/ab/liblda_old.so > $O/ab.log 2>&1 || { echo ab failed; tail -20 $O/ab.log; exit 1; }
tail -3 $O/ab.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lda_gpu.py tests/test_rowcodec_gpu.py tests/test_lda_pp_mp_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u scripts/bench_lda.py --docs 1000000 --topics 10000 --iters 5 > $O/k10k_rot.log 2>&1 || { echo rot failed; tail $O/k10k_rot.log; exit 1; }
tail -1 $O/k10k_rot.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('k10k rot', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
HARP_LDA_SAMPLER=sparse timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --strategy push_pull --local-server off --iters 5 > $O/k1k_sparse.log 2>&1 || { echo sparse failed; tail $O/k1k_sparse.log; exit 1; }
tail -1 $O/k1k_sparse.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('k1k sparse pp', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
