#!/bin/bash
# SYRK: off-diagonal-only timing of variant 0 vs variant 1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4p
timeout -k 10 300 python scripts/syrk_diag.py --modes 0,5,6,1 > gpurun_out/r4p/diag.log 2>&1 || { tail -20 gpurun_out/r4p/diag.log; exit 1; }
tail -1 gpurun_out/r4p/diag.log
