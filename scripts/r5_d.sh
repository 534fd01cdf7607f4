#!/bin/bash
# MF-SGD concurrency vs accuracy on the ML-10M gate (blocks per XCD), plus the new LDA K tests
set -o pipefail
O=gpurun_out/round5_d
mkdir -p $O
export PYTHONUNBUFFERED=1
for B in 16 32 64; do
  timeout -k 10 300 python -u scripts/ml10m_gate.py --device cuda --workers 2 --atomic 0 --blocks-per-xcd $B > $O/gate_b$B.json 2> $O/gate_b$B.err || { echo "gate b$B failed"; tail -20 $O/gate_b$B.err; exit 1; }
  tail -1 $O/gate_b$B.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('blocks', $B, d['test_rmse'], d['mean_epoch_s'])"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lda_gpu.py -k "conditional" \
  > $O/pytest_lda.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_lda.log; exit 1; }
tail -3 $O/pytest_lda.log
