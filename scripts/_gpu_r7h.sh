#!/bin/bash
# round-3: EM-GMM E-step with scalar-loaded whitening matrices, component-major R
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r7h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gmm_gpu.py -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|EM iter|Error" $O/pytest.log | tail -20
case $rc in 0|1) ;; *) exit $rc;; esac
for PPT in 1; do
for D in 8 16 32 64; do
  HARP_GMM_PPT=$PPT D=$D timeout -k 10 120 python scripts/probe_gmm.py > $O/probe_d${D}_p$PPT.log 2>&1 || { tail -3 $O/probe_d${D}_p$PPT.log; exit 1; }
  echo "ppt $PPT: $(grep '^{' $O/probe_d${D}_p$PPT.log)"
done
done
