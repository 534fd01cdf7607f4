#!/bin/bash
# round-3: fused look-ahead Householder reduction (one pass + one arrival per column) vs two-pass
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_eig_gpu.py -v -s --timeout 120 --timeout-method thread > $O/pytest_fused.log 2>&1
rc=$?; echo "pytest fused rc=$rc"; tail -3 $O/pytest_fused.log; grep eigvalsh $O/pytest_fused.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_eig_fused.py > $O/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat $O/probe.log
