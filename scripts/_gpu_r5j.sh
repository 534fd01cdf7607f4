#!/bin/bash
# round-2 final validation: GPU suite, smoke, default bench (all nested records), K-means-only kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5j
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5j/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r5j/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r5j/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5j/smoke.log 2>&1 || { tail -20 gpurun_out/r5j/smoke.log; exit 1; }
tail -1 gpurun_out/r5j/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r5j/bench.log 2>&1 || { tail -20 gpurun_out/r5j/bench.log; exit 1; }
grep '^{' gpurun_out/r5j/bench.log | tail -1 | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_km -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --sgd off --extras off > $GRAFT_REPO_ROOT/gpurun_out/r5j/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r5j/prof.log; exit 1; }
find /tmp/prof_km -name '*kernel_stats.csv' -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/r5j/kernel_stats.csv \;
grep '^{' $GRAFT_REPO_ROOT/gpurun_out/r5j/prof.log | tail -1 | cut -c1-200
