#!/bin/bash
# round-3 validation after the fused eigensolver and the one-slice SGD record: default bench
# (every nested record) + kernel stats of the bench (CSV; the full trace stays on the box)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8g
mkdir -p $O
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof8g -o bench -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 > $O/prof.log 2>&1
echo "prof rc=$?"
find /tmp/prof8g -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -25 $O/kernel_stats.csv | cut -c1-160
