#!/bin/bash
# dense LDA sampler phase split (diagnostic stamps build) at the 8-GPU share and at full size
set -o pipefail
O=gpurun_out/round5_r
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/lda_stamps.py --docs 125000 --strategy push_pull --local-server off --iters 3 > $O/share8.log 2>&1 || { echo share failed; tail $O/share8.log; exit 1; }
tail -1 $O/share8.log
HARP_LDA_SAMPLER=dense timeout -k 10 300 python -u scripts/lda_stamps.py --docs 1000000 --strategy push_pull --local-server off --iters 3 > $O/full.log 2>&1 || { echo full failed; tail $O/full.log; exit 1; }
tail -1 $O/full.log
