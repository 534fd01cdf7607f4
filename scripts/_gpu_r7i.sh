#!/bin/bash
# round-3: one-XCD symmetric eigensolver
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r7i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_eig_gpu.py -v -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|eigvalsh|Error|assert" $O/pytest.log | tail -30
exit $rc
