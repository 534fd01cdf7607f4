#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/syrk6
timeout -k 10 300 python scripts/syrk_diag.py > gpurun_out/syrk6/diag.log 2>&1 || { tail -20 gpurun_out/syrk6/diag.log; exit 1; }
tail -1 gpurun_out/syrk6/diag.log
