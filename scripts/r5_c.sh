#!/bin/bash
# W-only atomic write-back: gate + Netflix-shape epoch time; then the full bench (LDA headline = push-pull)
set -o pipefail
O=gpurun_out/round5_c
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_sgd_rank_placement_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for A in 1; do
  timeout -k 10 300 python -u scripts/ml10m_gate.py --device cuda --workers 2 --atomic $A > $O/gate_a$A.json 2> $O/gate_a$A.err || { echo "gate $A failed"; tail -20 $O/gate_a$A.err; exit 1; }
  tail -1 $O/gate_a$A.json | cut -c 180-420
done
for A in 1 0; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 3 --warmup 1 --points 1e7 --extras off --sgd on --sgd-atomic $A > $O/bench_sgd_a$A.json 2> $O/bench_sgd_a$A.err || { echo "bench $A failed"; tail -20 $O/bench_sgd_a$A.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_sgd_a$A.json'))['sgd'];print('atomic',$A,d['s_per_epoch'],d['epoch_s'],d['train_rmse'])"
done
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['sgd']['s_per_epoch'], d['pca']['s_per_pass'], d['lda']['tokens_per_sec'], d['lda'].get('local_server_alias'))"
