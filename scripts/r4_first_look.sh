#!/bin/bash
# round 4 first look: full GPU suite (no -x) + LDA push-pull layout diagnostic
mkdir -p gpurun_out/r5a
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5a/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u scripts/diag_lda_pp.py > gpurun_out/r5a/diag.log 2>&1
echo "diag rc=$?"
