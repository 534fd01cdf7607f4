#!/bin/bash
# round-3: where the LDA push-pull setup time goes at 3 gloo ranks sharing one GPU
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8q
mkdir -p $O
timeout -k 10 300 python -u scripts/probe_lda_setup.py 3 > $O/prof3.log 2>&1
rc=$?; echo "rc=$rc"; grep -v "Gloo\|socket\|amdgpu.ids" $O/prof3.log | head -45
