#!/bin/bash
# MF-CCD residual carry: GPU CCD tests, bench with resync 1 (reference schedule) vs 10
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4k
timeout -k 10 300 python -u -m pytest tests/test_ccd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4k/tests.log 2>&1 || { tail -30 gpurun_out/r4k/tests.log; exit 1; }
tail -1 gpurun_out/r4k/tests.log
for r in 10; do
  timeout -k 10 300 python scripts/bench_ccd.py --iters 5 --resync $r > gpurun_out/r4k/ccd_resync$r.log 2>&1 || { tail -20 gpurun_out/r4k/ccd_resync$r.log; exit 1; }
  grep '^{' gpurun_out/r4k/ccd_resync$r.log | tail -1 | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["residual_resync"], round(r["value"],4), [round(x,6) for x in r["train_rmse"]])'
done
