#!/bin/bash
mkdir -p gpurun_out/r4b4
timeout -k 10 300 python -u -m pytest tests/test_kmeans_gpu.py -q -k "wide" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4b4/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/bench_kmeans_wide.py 1e7 1000 1000 1,3,5,6 > gpurun_out/r4b4/kwide.log 2>&1
echo "rc=$?"
