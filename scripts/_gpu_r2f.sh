#!/bin/bash
# full gpu suite + headline bench + kernel-trace profile of the bench
set -o pipefail
mkdir -p gpurun_out/r2f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2f/pytest.log 2>&1 || { tail -40 gpurun_out/r2f/pytest.log; exit 1; }
tail -2 gpurun_out/r2f/pytest.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2f/bench.log 2>&1 || { tail -30 gpurun_out/r2f/bench.log; exit 1; }
tail -1 gpurun_out/r2f/bench.log | cut -c1-400
timeout -k 10 300 python bench.py --gpus 1 --points 1.25e7 --steps 20 --warmup 5 --sgd off > gpurun_out/r2f/bench_1.25e7.log 2>&1 || { tail -30 gpurun_out/r2f/bench_1.25e7.log; exit 1; }
tail -1 gpurun_out/r2f/bench_1.25e7.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2f/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r2f/prof.log 2>&1
echo prof rc=$?
