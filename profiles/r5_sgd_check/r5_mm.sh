#!/bin/bash
# MF-SGD bench record with and without the default kernel's XCD placement check (alternating, same box)
set -o pipefail
O=gpurun_out/round5_mm
mkdir -p $O
export PYTHONUNBUFFERED=1
for C in 1 0 1 0; do
  HARP_MF_CHECK_PLACEMENT=$C timeout -k 10 300 python -u bench.py --gpus 1 --steps 3 --warmup 1 --points 1e7 --extras off --sgd on > $O/sgd_chk$C.json 2> $O/sgd_chk$C.err || { echo "bench failed"; tail -20 $O/sgd_chk$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/sgd_chk$C.json'))['sgd'];print('check',$C,d['s_per_epoch'],d['epoch_s'])"
done
