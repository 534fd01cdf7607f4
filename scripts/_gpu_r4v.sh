#!/bin/bash
# K-means assign: refactored argmin (no spills) vs the committed tail-stage build (14 spills), same box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4v
for i in 1 2; do
  timeout -k 10 300 python scripts/kmeans_variant_ab.py 14 14 > gpurun_out/r4v/new$i.log 2>&1 || { tail -20 gpurun_out/r4v/new$i.log; exit 1; }
  echo "new: $(tail -1 gpurun_out/r4v/new$i.log)"
  HARP_KERNEL_LIB=$PWD/harp_amd/_native/libharp_kmeans_head.so timeout -k 10 300 python scripts/kmeans_variant_ab.py 14 14 > gpurun_out/r4v/head$i.log 2>&1 || { tail -20 gpurun_out/r4v/head$i.log; exit 1; }
  echo "head: $(tail -1 gpurun_out/r4v/head$i.log)"
done
