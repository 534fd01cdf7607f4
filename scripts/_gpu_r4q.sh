#!/bin/bash
# CCD rotation mode with the block kernels; LDA rotation / push-pull after the codec hook
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4q
timeout -k 10 300 python scripts/bench_ccd.py --iters 3 --mode rotation > gpurun_out/r4q/ccd_rot.log 2>&1 || { tail -20 gpurun_out/r4q/ccd_rot.log; exit 1; }
grep '^{' gpurun_out/r4q/ccd_rot.log | tail -1 | cut -c1-260
timeout -k 10 300 python scripts/bench_lda.py --iters 5 > gpurun_out/r4q/lda.log 2>&1 || { tail -20 gpurun_out/r4q/lda.log; exit 1; }
grep '^{' gpurun_out/r4q/lda.log | tail -1 | cut -c1-300
