#!/bin/bash
# round 5 first GPU pass: any-rank MF-SGD, placement check / placed kernel, LDA K%4 fused rows,
# the ML-10M gate at r=40 on the GPU, and the full bench
set -o pipefail
O=gpurun_out/round5_a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_sgd_rank_placement_gpu.py tests/test_sgd_mf_gpu.py tests/test_sgd_flow_gpu.py tests/test_lda_pp_mp_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python -u scripts/ml10m_gate.py --device cuda --workers 2 > $O/gate.json 2> $O/gate.err || { echo "gate failed"; tail -30 $O/gate.err; exit 1; }
cut -c 1-600 $O/gate.json
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cut -c 1-400 $O/bench.json
