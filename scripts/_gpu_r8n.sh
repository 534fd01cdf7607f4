#!/bin/bash
# round-3: MF-SGD GPU tests incl. the one-slice-per-rank test
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_sgd_mf_gpu.py -v --timeout 200 --timeout-method thread > $O/pytest_sgd.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_sgd.log; exit $rc
