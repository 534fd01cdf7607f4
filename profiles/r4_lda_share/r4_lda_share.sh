#!/bin/bash
# LDA push-pull at the 8-GPU rank share (docs / 8, full vocabulary) on one GPU: timing + kernel stats
mkdir -p gpurun_out/r4_lda
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > gpurun_out/r4_lda/share8.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_lda/prof -o run -- python3 scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > gpurun_out/r4_lda/prof.log 2>&1
echo "prof rc=$?"
