#!/bin/bash
# round-3: where the MF-SGD record's setup goes with 8 gloo ranks sharing one GPU (229 s in r8x)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8y
mkdir -p $O
HARP_BENCH_TRACE=1 timeout -k 10 600 python -u scripts/probe_sgd_setup.py 8 > $O/prof8.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; echo "hb $(grep -c rank $O/prof8.log)"; done
wait $pid; rc=$?; echo "rc=$rc"; grep -v "Gloo\|socket\|amdgpu.ids" $O/prof8.log | grep -v "^ " | head -60
