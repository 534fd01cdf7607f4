#!/bin/bash
# round-3: SMO 1024-thread forms up to 24k rows (fewer gather round trips)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_svm_gpu.py -v -s --timeout 250 --timeout-method thread > $O/pytest_svm.log 2>&1
rc=$?; echo "svm pytest rc=$rc"; grep -E "PASS|FAIL|device " $O/pytest_svm.log | tail -12
