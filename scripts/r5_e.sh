#!/bin/bash
# default concurrency cap on the ML-10M gate; Netflix-shape epoch time at the capped / uncapped block count;
# DAAL implicit ALS on ML-10M (Dim 100)
set -o pipefail
O=gpurun_out/round5_e
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/ml10m_gate.py --device cuda --workers 2 > $O/gate_default.json 2> $O/gate_default.err || { echo "gate failed"; tail -20 $O/gate_default.err; exit 1; }
tail -1 $O/gate_default.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['blocks_per_xcd'], d['test_rmse'], d['pass'], d['mean_epoch_s'])"
for B in 104 128; do
  timeout -k 10 300 python -u scripts/bench_sgd.py --epochs 10 --warmup 1 --blocks-per-xcd $B > $O/sgd_b$B.json 2> $O/sgd_b$B.err || { echo "sgd $B failed"; tail -20 $O/sgd_b$B.err; exit 1; }
  tail -1 $O/sgd_b$B.json | cut -c 1-300
done
timeout -k 10 600 python -u scripts/ml10m_gate.py --device cuda --workers 2 --als > $O/als.json 2> $O/als.err || { echo "als failed"; tail -20 $O/als.err; exit 1; }
tail -1 $O/als.json | cut -c 1-700
