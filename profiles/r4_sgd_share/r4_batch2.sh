#!/bin/bash
# wide K-means (swizzle fix) variants; MF-SGD prefetch-distance variants at full size and the
# 8-GPU share; LDA push-pull 8-share with the sparse sampler forced
mkdir -p gpurun_out/r4b2
timeout -k 10 200 python -u scripts/bench_kmeans_wide.py 1e7 1000 1000 1,2,3,4 > gpurun_out/r4b2/kwide.log 2>&1 || exit $?
for v in 0 2 3; do
  timeout -k 10 200 python -u scripts/bench_sgd.py --epochs 10 --chunk 0 --variant $v >> gpurun_out/r4b2/sgd_full.log 2>&1 || exit $?
  timeout -k 10 200 python -u scripts/bench_sgd.py --epochs 10 --chunk 0 --variant $v --users 60024 --ratings 12560063 >> gpurun_out/r4b2/sgd_share8.log 2>&1 || exit $?
  timeout -k 10 200 python -u scripts/bench_sgd.py --epochs 10 --chunk 0 --variant $v --users 60024 --ratings 12560063 --slices 2 >> gpurun_out/r4b2/sgd_share8_s2.log 2>&1 || exit $?
done
HARP_LDA_SAMPLER=sparse timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > gpurun_out/r4b2/lda_share8_sparse.log 2>&1
echo "rc=$?"
