#!/bin/bash
# round-2 first GPU check: gpu tests, bench, kernel-trace stats
set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1 || { tail -30 gpurun_out/r2a/pytest.log; exit 1; }
tail -3 gpurun_out/r2a/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2a/bench.log 2>&1 || { tail -30 gpurun_out/r2a/bench.log; exit 1; }
tail -1 gpurun_out/r2a/bench.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2a/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r2a/prof.log 2>&1
echo prof rc=$?
