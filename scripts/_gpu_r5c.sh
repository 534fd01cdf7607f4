#!/bin/bash
# LDA push-pull single-worker local server: LDA GPU tests + bench (local server on / off)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
timeout -k 10 300 python -u -m pytest tests/test_lda_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5c/tests.log 2>&1 || { tail -30 gpurun_out/r5c/tests.log; exit 1; }
tail -1 gpurun_out/r5c/tests.log
timeout -k 10 300 python bench.py --points 1e6 --steps 2 --warmup 1 --sgd off --extras on --pca-n 4.8e5 > gpurun_out/r5c/bench.log 2>&1 || { tail -20 gpurun_out/r5c/bench.log; exit 1; }
grep '^{' gpurun_out/r5c/bench.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['lda'])"
