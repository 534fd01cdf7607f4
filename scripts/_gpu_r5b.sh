#!/bin/bash
# LDA push-pull vs rotation kernel stats (1M docs x 1M vocab x 1000 topics, 1 GPU)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5b
for st in push_pull rotation; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$st -o run -- python $GRAFT_REPO_ROOT/scripts/bench_lda.py --iters 3 --strategy $st > $GRAFT_REPO_ROOT/gpurun_out/r5b/$st.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r5b/$st.log; exit 1; }
  grep '^{' $GRAFT_REPO_ROOT/gpurun_out/r5b/$st.log | tail -1 | cut -c1-120
  find /tmp/prof_$st -name '*kernel_stats.csv' -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/r5b/kernel_stats_$st.csv \;
done
ls -la $GRAFT_REPO_ROOT/gpurun_out/r5b
