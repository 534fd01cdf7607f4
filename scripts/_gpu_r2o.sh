#!/bin/bash
# identity / overwrite fast paths of the planned push-pull: LDA push-pull + K-means push_pull, 1 GPU
set -o pipefail
mkdir -p gpurun_out/r2o
timeout -k 10 300 python -u -m pytest tests/test_lda_gpu.py tests/test_plans.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2o/pytest.log 2>&1 || { tail -30 gpurun_out/r2o/pytest.log; exit 1; }
tail -1 gpurun_out/r2o/pytest.log
timeout -k 10 300 python scripts/bench_lda.py --strategy push_pull --iters 5 > gpurun_out/r2o/lda_pp.log 2>&1 || { tail -20 gpurun_out/r2o/lda_pp.log; exit 1; }
tail -1 gpurun_out/r2o/lda_pp.log | cut -c1-200
timeout -k 10 300 python scripts/bench_lda.py --strategy rotation --iters 5 > gpurun_out/r2o/lda_rot.log 2>&1 || { tail -20 gpurun_out/r2o/lda_rot.log; exit 1; }
tail -1 gpurun_out/r2o/lda_rot.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --strategy push_pull --sgd off > gpurun_out/r2o/km_pp.log 2>&1 || { tail -20 gpurun_out/r2o/km_pp.log; exit 1; }
tail -1 gpurun_out/r2o/km_pp.log | cut -c1-160
