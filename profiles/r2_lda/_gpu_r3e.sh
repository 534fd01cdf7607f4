#!/bin/bash
# LDA at K=10,000 and K=2000 with workgroup LDS word-row deltas (+ K=1000 regression check)
set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_lda_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e/pytest.log 2>&1; tail -1 gpurun_out/r3e/pytest.log
for k in 10000 2000 1000; do
  for rep in 1 2; do
    timeout -k 10 300 python scripts/bench_lda.py --iters 3 --topics $k > gpurun_out/r3e/k${k}_$rep.log 2>&1 || { tail -5 gpurun_out/r3e/k${k}_$rep.log; exit 1; }
    python -c "import json; r=json.loads(open('gpurun_out/r3e/k${k}_$rep.log').read().strip().splitlines()[-1]); print('K=$k', $rep, round(r['s_per_iter'],5), r['loglik_end'])"
  done
done
