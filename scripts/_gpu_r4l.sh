#!/bin/bash
# MF-CCD kernel-trace profile (Netflix shape, rank 120)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4l
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4l/prof -o run -- python $GRAFT_REPO_ROOT/scripts/bench_ccd.py --iters 2 > $GRAFT_REPO_ROOT/gpurun_out/r4l/ccd.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4l/ccd.log; exit 1; }
grep '^{' $GRAFT_REPO_ROOT/gpurun_out/r4l/ccd.log | tail -1 | cut -c1-300
