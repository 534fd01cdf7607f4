#!/bin/bash
# persistent cooperative XCD SGD launch: numerics, then the 8-GPU share / full Netflix, off vs on
set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 200 python -u -m pytest tests/test_sgd_mf_gpu.py -x -q --timeout 60 --timeout-method thread -k "persistent or xcd" > gpurun_out/r3g/pytest.log 2>&1 || { tail -30 gpurun_out/r3g/pytest.log; exit 1; }
tail -1 gpurun_out/r3g/pytest.log
for mode in off on; do
  HARP_SGD_PERSISTENT=$mode timeout -k 10 200 python bench.py --points 1e6 --centroids 1000 --steps 2 --warmup 1 --sgd on --sgd-ratings 12560063 --sgd-slices 16 --sgd-epochs 20 --sgd-warmup 3 > gpurun_out/r3g/s16_$mode.log 2>&1 || { tail -20 gpurun_out/r3g/s16_$mode.log; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/r3g/s16_$mode.log').read().strip().splitlines()[-1])['sgd']; print('12.5M/16 $mode', r['s_per_epoch'], r['train_rmse'])"
  HARP_SGD_PERSISTENT=$mode timeout -k 10 200 python bench.py --points 1e6 --centroids 1000 --steps 2 --warmup 1 --sgd on --sgd-epochs 10 > gpurun_out/r3g/full_$mode.log 2>&1 || { tail -20 gpurun_out/r3g/full_$mode.log; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/r3g/full_$mode.log').read().strip().splitlines()[-1])['sgd']; print('100M $mode', r['s_per_epoch'], r['train_rmse'])"
done
