#!/bin/bash
# XCD-contiguous chunk order in the label bucketing scatter: numerics + bench + kernel stats
set -o pipefail
mkdir -p gpurun_out/r2u
timeout -k 10 300 python -u -m pytest tests/test_kmeans_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2u/pytest.log 2>&1; tail -1 gpurun_out/r2u/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sgd off > gpurun_out/r2u/bench.log 2>&1 || { tail -20 gpurun_out/r2u/bench.log; exit 1; }
tail -1 gpurun_out/r2u/bench.log | cut -c1-110
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_u -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --sgd off > $GRAFT_REPO_ROOT/gpurun_out/r2u/prof.log 2>&1
cd $GRAFT_REPO_ROOT && python scripts/rocpd_summary.py /tmp/prof_u/run_results.db --top 8 --out gpurun_out/r2u/kernel_stats.json > /dev/null && python -c "
import json
d=json.load(open('gpurun_out/r2u/kernel_stats.json'))
for k in d['top']: print(round(k['avg_us'],1), k['calls'], k['kernel'][:60])"
