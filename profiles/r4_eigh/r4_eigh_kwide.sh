#!/bin/bash
# eigenvectors (D&C) + wide-row K-means: tests, timing, kernel stats
mkdir -p gpurun_out/r5c
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_eig_gpu.py tests/test_kmeans_gpu.py tests/test_coop_contention_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5c/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/prof_eigh.py > gpurun_out/r5c/time.log 2>&1 || exit $?
timeout -k 10 120 python -u scripts/bench_kmeans_wide.py > gpurun_out/r5c/kwide.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5c/prof -o run -- python3 scripts/prof_eigh.py > gpurun_out/r5c/prof.log 2>&1
echo "prof rc=$?"
