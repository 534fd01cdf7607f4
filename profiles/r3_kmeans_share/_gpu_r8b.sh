#!/bin/bash
# round-3: K-means per-rank shares of the 2/4/8-GPU runs on one GPU (strong-scaling overhead) + kernel trace at the 8-GPU share
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8b
mkdir -p $O
for N in 1e8 5e7 2.5e7 1.25e7; do
  timeout -k 10 200 python bench.py --points $N --sgd off --extras off --steps 20 --warmup 3 > $O/share_$N.log 2>&1
  rc=$?; echo "N=$N rc=$rc $(grep '^{' $O/share_$N.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["median_s_per_iter"], r["phase_ms_per_iter"])')"
  [ $rc -eq 0 ] || exit $rc
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o share8 -- python $GRAFT_REPO_ROOT/bench.py --points 1.25e7 --sgd off --extras off --steps 20 --warmup 3 > $O/prof.log 2>&1
echo "prof rc=$?"
find $O/prof -name '*stats*' | head
