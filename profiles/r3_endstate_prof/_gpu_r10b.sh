#!/bin/bash
# round-3 end-state kernel profile: rocprofv3 kernel trace + stats of the default bench (all nested records)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r10b
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; grep '^{' $O/bench.log | cut -c1-200
python3 scripts/rocpd_summary.py $O/prof/run_results.db --out $O/kernels.json --top 40 > $O/summary.txt 2>&1; echo "summary rc=$?"
rm -rf $O/prof
head -30 $O/summary.txt
exit $rc
