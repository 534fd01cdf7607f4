#!/bin/bash
# CCD with int32 residual permutations: GPU CCD tests + bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5i
timeout -k 10 300 python -u -m pytest tests/test_ccd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5i/tests.log 2>&1 || { tail -30 gpurun_out/r5i/tests.log; exit 1; }
tail -1 gpurun_out/r5i/tests.log
timeout -k 10 300 python scripts/bench_ccd.py --iters 5 > gpurun_out/r5i/ccd.log 2>&1 || { tail -20 gpurun_out/r5i/ccd.log; exit 1; }
grep '^{' gpurun_out/r5i/ccd.log | tail -1 | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["value"],4), [round(x,6) for x in r["train_rmse"]])'
