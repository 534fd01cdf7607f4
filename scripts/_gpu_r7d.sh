#!/bin/bash
# round-3: SMO with the diagonal in LDS, register publish, prefetched alphas
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r7d
timeout -k 10 400 python -u -m pytest tests/test_svm_gpu.py tests/test_ctypes_signatures.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r7d/pytest_svm.log 2>&1
rc=$?; echo "svm pytest rc=$rc"; grep -E "PASS|FAIL|device|Error|assert" gpurun_out/r7d/pytest_svm.log | tail -30
exit $rc
