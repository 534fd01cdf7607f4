#!/bin/bash
# round-3: the P-rank SGD shares rehearsed with the rank's USER count (users are partitioned
# over ranks, so a rank's W holds 1/P of the users), variants 0 and 2; kernel trace of the
# 8-rank share
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r7c
for P in 8 4 2; do
  U=$(( (480189 + P - 1) / P )); N=$(( (100480507 + P - 1) / P )); S=$(( 2 * P ))
  for v in 0 2; do
    timeout -k 10 200 python scripts/bench_sgd.py --users $U --ratings $N --slices $S --epochs 10 --variant $v --chunk 0 > gpurun_out/r7c/share${P}_v$v.log 2>&1 || { echo "share$P v$v failed"; tail -5 gpurun_out/r7c/share${P}_v$v.log; exit 1; }
    echo "P=$P share v$v: $(grep '^{' gpurun_out/r7c/share${P}_v$v.log | cut -c1-250)"
  done
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof7c -o run -- python $GRAFT_REPO_ROOT/scripts/bench_sgd.py --users 60024 --ratings 12560063 --slices 16 --epochs 5 --variant 0 --chunk 0 > $GRAFT_REPO_ROOT/gpurun_out/r7c/prof.log 2>&1 || { echo "prof failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/r7c/prof.log; exit 1; }
find /tmp/prof7c -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/r7c/kernel_stats.csv \;
find /tmp/prof7c -name "*kernel_trace.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/r7c/kernel_trace.csv \;
ls -la $GRAFT_REPO_ROOT/gpurun_out/r7c/
head -12 $GRAFT_REPO_ROOT/gpurun_out/r7c/kernel_stats.csv | cut -c1-200
