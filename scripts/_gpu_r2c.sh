#!/bin/bash
# GPU tests + 1-GPU bench for every K-means sync strategy (push_pull must be within ~5 ms of allreduce)
set -o pipefail
mkdir -p gpurun_out/r2c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c/pytest.log 2>&1 || { tail -40 gpurun_out/r2c/pytest.log; exit 1; }
tail -3 gpurun_out/r2c/pytest.log
for s in allreduce regroup_allgather bcast_reduce push_pull rotation; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --strategy $s --sgd off > gpurun_out/r2c/bench_$s.log 2>&1 || { tail -20 gpurun_out/r2c/bench_$s.log; exit 1; }
  tail -1 gpurun_out/r2c/bench_$s.log | cut -c1-200
done
