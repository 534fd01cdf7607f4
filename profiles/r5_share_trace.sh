#!/bin/bash
# LDA 8-GPU share sweep (push-pull, one GPU): kernel trace + stats, to split the sweep's wall time
set -o pipefail
O=gpurun_out/round5_share_trace
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > $O/share.log 2>&1 || { echo "trace failed"; tail -20 $O/share.log; exit 1; }
tail -1 $O/share.log
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
find $O/trace -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/kernel_trace.csv
rm -rf $O/trace
echo done
