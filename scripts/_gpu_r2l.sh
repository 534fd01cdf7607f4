#!/bin/bash
# adaptive SGD stream chunk: SGD GPU tests, the 8-GPU per-rank share with 2 / 16 slices, full Netflix 1 GPU
set -o pipefail
mkdir -p gpurun_out/r2l
timeout -k 10 300 python -u -m pytest tests/test_sgd_mf_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2l/pytest.log 2>&1 || { tail -30 gpurun_out/r2l/pytest.log; exit 1; }
tail -1 gpurun_out/r2l/pytest.log
for s in 2 16; do
  timeout -k 10 300 python bench.py --points 1e6 --centroids 1000 --steps 2 --warmup 1 --sgd on --sgd-ratings 12560063 --sgd-slices $s --sgd-epochs 20 --sgd-warmup 3 > gpurun_out/r2l/sgd_s$s.log 2>&1 || { tail -20 gpurun_out/r2l/sgd_s$s.log; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/r2l/sgd_s$s.log').read().strip().splitlines()[-1])['sgd']; print('12.5M slices=$s', r['s_per_epoch'], r['updates_per_sec'], r['train_rmse'])"
done
timeout -k 10 300 python bench.py --points 1e6 --centroids 1000 --steps 2 --warmup 1 --sgd on --sgd-epochs 10 > gpurun_out/r2l/sgd_full.log 2>&1 || { tail -20 gpurun_out/r2l/sgd_full.log; exit 1; }
python -c "import json; r=json.loads(open('gpurun_out/r2l/sgd_full.log').read().strip().splitlines()[-1])['sgd']; print('100M', r['s_per_epoch'], r['updates_per_sec'], r['train_rmse'])"
