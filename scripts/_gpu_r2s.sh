#!/bin/bash
# A/B on one box: K-means assign built with / without IEEE mode (no NaN canonicalisation in the argmin)
set -o pipefail
mkdir -p gpurun_out/r2s
for lib in base noieee base noieee; do
  if [ $lib = noieee ]; then export HARP_KERNEL_LIB=$PWD/alt_libs/libharp_kernels_noieee.so; else unset HARP_KERNEL_LIB; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sgd off > gpurun_out/r2s/bench_$lib.log 2>&1 || { tail -20 gpurun_out/r2s/bench_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/r2s/bench_$lib.log | cut -c1-110)"
done
HARP_KERNEL_LIB=$PWD/alt_libs/libharp_kernels_noieee.so timeout -k 10 300 python -u -m pytest tests/test_kmeans_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s/pytest.log 2>&1; tail -1 gpurun_out/r2s/pytest.log
