#!/bin/bash
# bench with the nested SGD record (1 GPU) + 2-rank gloo rehearsal of the self-spawn path on one GPU
set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --metrics-jsonl gpurun_out/r2b/km.jsonl > gpurun_out/r2b/bench.log 2>&1 || { tail -30 gpurun_out/r2b/bench.log; exit 1; }
tail -1 gpurun_out/r2b/bench.log
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --points 2e7 --steps 5 --warmup 2 --sgd on --sgd-ratings 20000000 > gpurun_out/r2b/bench_gloo2.log 2>&1 || { tail -30 gpurun_out/r2b/bench_gloo2.log; exit 1; }
tail -1 gpurun_out/r2b/bench_gloo2.log
