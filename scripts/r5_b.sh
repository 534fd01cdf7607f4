#!/bin/bash
# atomic (no-lost-update) SGD write-back: tests, ML-10M gate A/B, Netflix-shape epoch time A/B
set -o pipefail
O=gpurun_out/round5_b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_sgd_rank_placement_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
grep -E "sse initial" $O/pytest.log || true
for A in 1 0; do
  timeout -k 10 300 python -u scripts/ml10m_gate.py --device cuda --workers 2 --atomic $A > $O/gate_a$A.json 2> $O/gate_a$A.err || { echo "gate $A failed"; tail -20 $O/gate_a$A.err; exit 1; }
  tail -1 $O/gate_a$A.json | cut -c 1-420
done
timeout -k 10 300 python -u scripts/ml10m_gate.py --device cuda --workers 2 --atomic 0 --blocks-per-xcd 8 --chunk 64 > $O/gate_a0_b8.json 2> $O/gate_a0_b8.err || { echo "gate b8 failed"; exit 1; }
tail -1 $O/gate_a0_b8.json | cut -c 1-420
for A in 0 1; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 3 --warmup 1 --points 1e7 --extras off --sgd on --sgd-atomic $A > $O/bench_sgd_a$A.json 2> $O/bench_sgd_a$A.err || { echo "bench $A failed"; tail -20 $O/bench_sgd_a$A.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_sgd_a$A.json'))['sgd'];print('atomic',$A,d['s_per_epoch'],d['epoch_s'],d['train_rmse'])"
done
