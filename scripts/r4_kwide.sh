#!/bin/bash
mkdir -p gpurun_out/r4_kwide
timeout -k 10 200 python -u scripts/bench_kmeans_wide.py 1e7 1000 1000 1,2,3,4 > gpurun_out/r4_kwide/v.log 2>&1
echo "rc=$?"
