#!/bin/bash
mkdir -p gpurun_out/r4b6
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kmeans_gpu.py tests/test_rowcodec_gpu.py tests/test_lda_gpu.py -q -k "wide or lda or rowcodec" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4b6/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/bench_kmeans_wide.py 1e7 1000 1000 5,9 > gpurun_out/r4b6/kwide.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/bench_kmeans_wide.py 1e7 1000 512 5,9 > gpurun_out/r4b6/kwide_d512.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/bench_kmeans_wide.py 1e6 10000 1000 5,9 > gpurun_out/r4b6/kwide_k1e4.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > gpurun_out/r4b6/lda_share8_fused.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-include-regex "lda_cgs" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d gpurun_out/r4b6/pmc_lda -o run -- python3 scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 2 > gpurun_out/r4b6/pmc_lda.log 2>&1
echo "rc=$?"
du -sh gpurun_out/r4b6
