#!/bin/bash
# round-3: MF-SGD W-prefetch variant (2) — exactness tests and the 8-GPU-share A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r7a
timeout -k 10 300 python -u -m pytest tests/test_sgd_mf_gpu.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r7a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|rmse" gpurun_out/r7a/pytest.log | tail -30
case $rc in 0|1) ;; *) exit $rc;; esac
for v in 0 2 0 2; do
  timeout -k 10 200 python scripts/bench_sgd.py --ratings 12560063 --slices 16 --epochs 10 --variant $v --chunk 0 > gpurun_out/r7a/share_v$v.log 2>&1 || { echo "share v$v failed"; tail -5 gpurun_out/r7a/share_v$v.log; exit 1; }
  echo "8-share v$v: $(grep '^{' gpurun_out/r7a/share_v$v.log | cut -c1-250)"
done
for v in 0 2; do
  timeout -k 10 200 python scripts/bench_sgd.py --ratings 25120126 --slices 8 --epochs 10 --variant $v --chunk 0 > gpurun_out/r7a/share4_v$v.log 2>&1 || { echo "share4 v$v failed"; exit 1; }
  echo "4-share v$v: $(grep '^{' gpurun_out/r7a/share4_v$v.log | cut -c1-250)"
done
