#!/bin/bash
# MF-SGD per-step host overhead: the 8-GPU per-rank share (12.5M ratings) on one GPU with
# 2 vs 16 slices (16 = the sub-steps per epoch of an 8-rank, 2-slice rotation)
set -o pipefail
mkdir -p gpurun_out/r2k
for s in 2 16; do
  timeout -k 10 300 python bench.py --points 1e6 --centroids 1000 --steps 2 --warmup 1 --sgd on --sgd-ratings 12560063 --sgd-slices $s --sgd-epochs 20 --sgd-warmup 3 > gpurun_out/r2k/sgd_s$s.log 2>&1 || { tail -20 gpurun_out/r2k/sgd_s$s.log; exit 1; }
  python -c "import json,sys; r=json.loads(open('gpurun_out/r2k/sgd_s$s.log').read().strip().splitlines()[-1])['sgd']; print('slices=$s', r['s_per_epoch'], r['updates_per_sec'])"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2k/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --points 1e6 --centroids 1000 --steps 2 --warmup 1 --sgd on --sgd-ratings 12560063 --sgd-slices 16 --sgd-epochs 5 --sgd-warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r2k/prof.log 2>&1
echo prof rc=$?
