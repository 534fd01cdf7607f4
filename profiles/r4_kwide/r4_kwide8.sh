#!/bin/bash
# wide K-means: 8-wave (2 per SIMD) tile (variant 6) vs the 4-wave default (5)
mkdir -p gpurun_out/r4w
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kmeans_gpu.py -q -k wide --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4w/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/bench_kmeans_wide.py 1e7 1000 1000 5,6,5,6 > gpurun_out/r4w/kwide.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/bench_kmeans_wide.py 1e7 1000 512 5,6 > gpurun_out/r4w/kwide_d512.log 2>&1
echo "bench rc=$?"
