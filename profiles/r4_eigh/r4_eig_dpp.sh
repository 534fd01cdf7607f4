#!/bin/bash
# DPP fp64 wave sums in the eigensolver and D&C kernels: tests + timings + phases
mkdir -p gpurun_out/r4j
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_eig_gpu.py tests/test_coop_contention_gpu.py tests/test_linalg_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4j/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/probe_eig_phases.py 500 1000 1536 > gpurun_out/r4j/phases.log 2>&1 || exit $?
timeout -k 10 120 python -u scripts/prof_eigh.py 1000 > gpurun_out/r4j/time.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r4j/prof -o run -- python3 scripts/prof_eigh.py 1000 > gpurun_out/r4j/prof.log 2>&1
echo "prof rc=$?"
