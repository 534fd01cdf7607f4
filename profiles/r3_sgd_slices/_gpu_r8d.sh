#!/bin/bash
# round-3: MF-SGD rank shares with one H slice per rank (S = 1: 8 launches per slice step,
# half the launches per epoch) vs two (S = 2, the default), the rank's own users
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8d
mkdir -p $O
for P in 8 4 2; do
  U=$(( (480189 + P - 1) / P )); N=$(( (100480507 + P - 1) / P ))
  for S in 1 2; do
    timeout -k 10 200 python scripts/bench_sgd.py --users $U --ratings $N --slices $(( S * P )) --epochs 10 --chunk 0 > $O/share${P}_s$S.log 2>&1 || { echo "share$P S$S failed"; tail -5 $O/share${P}_s$S.log; exit 1; }
    echo "P=$P S=$S: $(grep '^{' $O/share${P}_s$S.log | cut -c1-220)"
  done
done
