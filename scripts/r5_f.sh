#!/bin/bash
# sparse doc-span sampler with fused parameter-server rows: tests, full-size and 8-share sweeps
set -o pipefail
O=gpurun_out/round5_f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lda_pp_mp_gpu.py tests/test_rowcodec_gpu.py tests/test_lda_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_lda.py --docs 1e6 --strategy push_pull --local-server off --iters 5 > $O/full.log 2>&1 || { echo full failed; tail $O/full.log; exit 1; }
tail -1 $O/full.log | cut -c 1-600
timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > $O/share8.log 2>&1 || { echo share failed; tail $O/share8.log; exit 1; }
tail -1 $O/share8.log | cut -c 1-600
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_sgd_rank_placement_gpu.py -k "cap or model_any" -s \
  > $O/pytest_cap.log 2>&1 || { echo "cap pytest failed"; tail -30 $O/pytest_cap.log; exit 1; }
grep -E "^cap|passed|failed" $O/pytest_cap.log | tail -3
timeout -k 10 600 python -u scripts/ml10m_gate.py --device cuda --workers 2 --als > $O/als.json 2> $O/als.err || { echo "als failed"; tail -5 $O/als.err; exit 1; }
tail -1 $O/als.json | cut -c 1-500
