#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for LF in 3; do
  echo "load flavor $LF"
  HARP_EIG_LOAD=$LF timeout -k 10 200 python -u -m pytest tests/test_eig_gpu.py -q -s --timeout 120 --timeout-method thread 2>&1 | grep -E "eigvalsh|passed|failed"
  HARP_EIG_LOAD=$LF STAMPS=1 timeout -k 10 100 python scripts/probe_eig_nb.py 2>&1 | grep stamp_cycles | cut -c1-300
done
