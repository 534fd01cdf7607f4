#!/bin/bash
# round-3: eigensolver GPU tests after removing the unused KU forms
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r9a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_eig_gpu.py tests/test_partial_results.py -q -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 $O/pytest.log; grep eigvalsh $O/pytest.log; exit $rc
