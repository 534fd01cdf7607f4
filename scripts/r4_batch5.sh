#!/bin/bash
mkdir -p gpurun_out/r4b5
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kmeans_gpu.py tests/test_lda_gpu.py tests/test_rowcodec_gpu.py -q -k "wide or lda or rowcodec" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4b5/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/bench_kmeans_wide.py 1e7 1000 1000 5,7,8 > gpurun_out/r4b5/kwide.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > gpurun_out/r4b5/lda_share8_u8.log 2>&1 || exit $?
HARP_LDA_NDK8=0 timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > gpurun_out/r4b5/lda_share8_u16.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/r4b5/pmc_v5 -o run -- python3 scripts/bench_kmeans_wide.py 2e6 1000 1000 5 > gpurun_out/r4b5/pmc_v5.log 2>&1
echo "rc=$?"
