#!/bin/bash
# round-2 validation after the SGD chunk / push-pull changes: gpu suite, bench (+SGD record), kernel-trace profile
set -o pipefail
mkdir -p gpurun_out/r2q
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2q/pytest.log 2>&1 || { tail -40 gpurun_out/r2q/pytest.log; exit 1; }
tail -1 gpurun_out/r2q/pytest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r2q/bench.log 2>&1 || { tail -30 gpurun_out/r2q/bench.log; exit 1; }
tail -1 gpurun_out/r2q/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_q -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r2q/prof.log 2>&1
echo prof rc=$?
cd $GRAFT_REPO_ROOT && python scripts/rocpd_summary.py /tmp/prof_q/run_results.db --top 20 --out gpurun_out/r2q/kernel_stats.json > /dev/null && cp /tmp/prof_q/run_kernel_stats.csv gpurun_out/r2q/ 2>/dev/null; ls gpurun_out/r2q
