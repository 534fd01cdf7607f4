#!/bin/bash
# MF-SGD bench record placement check at the block end vs off
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sgd_rank_placement_gpu.py tests/test_sgd_mf_gpu.py tests/test_coop_contention_gpu.py > gpurun_out/round5_nn_pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/round5_nn_pytest.log; exit 1; }
tail -1 gpurun_out/round5_nn_pytest.log
O=gpurun_out/round5_nn
mkdir -p $O
export PYTHONUNBUFFERED=1
for C in 1 0 1 0; do
  HARP_MF_CHECK_PLACEMENT=$C timeout -k 10 300 python -u bench.py --gpus 1 --steps 3 --warmup 1 --points 1e7 --extras off --sgd on > $O/sgd_chk$C.json 2> $O/sgd_chk$C.err || { echo "bench failed"; tail -20 $O/sgd_chk$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/sgd_chk$C.json'))['sgd'];print('check',$C,d['s_per_epoch'],d['epoch_s'])"
done
