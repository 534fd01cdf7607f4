#!/bin/bash
# hot-item replica rows for MF-SGD: tests, then full Netflix-shape (1 GPU) and the 8-GPU share, replicas on / off
set -o pipefail
mkdir -p gpurun_out/r2p
timeout -k 10 300 python -u -m pytest tests/test_sgd_mf_gpu.py -q -s --timeout 120 --timeout-method thread > gpurun_out/r2p/pytest.log 2>&1 || true
grep "sse initial" gpurun_out/r2p/pytest.log; tail -1 gpurun_out/r2p/pytest.log
for hr in 32 0; do
  HARP_SGD_HOT_REPLICAS=$hr timeout -k 10 300 python bench.py --points 1e6 --centroids 1000 --steps 2 --warmup 1 --sgd on --sgd-epochs 10 > gpurun_out/r2p/full_h$hr.log 2>&1 || { tail -20 gpurun_out/r2p/full_h$hr.log; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/r2p/full_h$hr.log').read().strip().splitlines()[-1])['sgd']; print('100M hot=$hr', r['s_per_epoch'], r['updates_per_sec'], r['train_rmse'])"
  HARP_SGD_HOT_REPLICAS=$hr timeout -k 10 300 python bench.py --points 1e6 --centroids 1000 --steps 2 --warmup 1 --sgd on --sgd-ratings 12560063 --sgd-slices 16 --sgd-epochs 20 --sgd-warmup 3 > gpurun_out/r2p/s16_h$hr.log 2>&1 || { tail -20 gpurun_out/r2p/s16_h$hr.log; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/r2p/s16_h$hr.log').read().strip().splitlines()[-1])['sgd']; print('12.5M/16 hot=$hr', r['s_per_epoch'], r['updates_per_sec'], r['train_rmse'])"
done
