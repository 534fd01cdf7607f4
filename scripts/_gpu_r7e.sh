#!/bin/bash
# round-3: cooperative multi-CU SMO — exactness vs the one-CU kernel, per-step timings
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r7e
timeout -k 10 500 python -u -m pytest tests/test_svm_gpu.py tests/test_ctypes_signatures.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r7e/pytest_svm.log 2>&1
rc=$?; echo "svm pytest rc=$rc"; grep -E "PASS|FAIL|device|Error|assert" gpurun_out/r7e/pytest_svm.log | tail -30
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python scripts/probe_svm_coop.py > gpurun_out/r7e/probe.log 2>&1; rc2=$?
cat gpurun_out/r7e/probe.log | grep '^{'
exit $rc2
