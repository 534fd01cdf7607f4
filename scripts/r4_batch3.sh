#!/bin/bash
# LDA 8-share: sparse sampler workgroup size; wide K-means PMC; SGD tests after cleanup
mkdir -p gpurun_out/r4b3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sgd_mf_gpu.py tests/test_sgd_flow_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4b3/sgd_tests.log 2>&1
rc=$?; echo "sgd tests rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in 1 2; do
  HARP_LDA_SAMPLER=sparse HARP_LDA_SPARSE_WAVES=$w timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > gpurun_out/r4b3/lda_sparse_w$w.log 2>&1 || exit $?
done
for v in 1 3; do
  HARP_KMEANS_WIDE_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/r4b3/pmc_v$v -o run -- python3 scripts/bench_kmeans_wide.py 2e6 1000 1000 $v > gpurun_out/r4b3/pmc_v$v.log 2>&1 || exit $?
done
echo done
