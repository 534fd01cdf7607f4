#!/bin/bash
# one-pass gather-sum for rows wider than 256 columns vs the 256-column slices (r4_kwide)
set -o pipefail
out=gpurun_out/r4rsw
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kmeans_gpu.py > $out/pytest.log 2>&1 || exit $?
for r in 1 2; do
  for sl in 1024 256; do
    HARP_ROWSUM_SLICE=$sl timeout -k 10 300 python -u scripts/bench_kmeans_wide.py 1e7 1000 1000 > $out/d1000_slice${sl}_$r.log 2>&1 || exit $?
    HARP_ROWSUM_SLICE=$sl timeout -k 10 300 python -u scripts/bench_kmeans_wide.py 1e7 1000 512 > $out/d512_slice${sl}_$r.log 2>&1 || exit $?
  done
done
