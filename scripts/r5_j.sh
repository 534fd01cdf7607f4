#!/bin/bash
set -o pipefail
O=gpurun_out/round5_j
mkdir -p $O
timeout -k 10 300 python -u scripts/lda_ab_det.py scripts/ab/liblda_old.so > $O/ab.log 2>&1; rc=$?
tail -5 $O/ab.log
exit $rc
