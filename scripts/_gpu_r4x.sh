#!/bin/bash
# round-2 validation after the CCD / ALS / K-means spill changes: GPU suite, smoke, bench, bench kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4x
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4x/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r4x/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4x/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4x/smoke.log 2>&1 || { tail -20 gpurun_out/r4x/smoke.log; exit 1; }
tail -1 gpurun_out/r4x/smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r4x/bench.log 2>&1 || { tail -20 gpurun_out/r4x/bench.log; exit 1; }
grep '^{' gpurun_out/r4x/bench.log | tail -1 | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4x/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r4x/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4x/prof.log; exit 1; }
grep '^{' $GRAFT_REPO_ROOT/gpurun_out/r4x/prof.log | tail -1 | cut -c1-200
