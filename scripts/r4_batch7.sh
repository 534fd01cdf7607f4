#!/bin/bash
mkdir -p gpurun_out/r4b7
timeout -k 10 400 python -u -m pytest tests/test_rowcodec_gpu.py tests/test_lda_gpu.py tests/test_lda_pp_mp_gpu.py -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r4b7/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 3 0; do
  HARP_LDA_VARIANT=$v timeout -k 10 300 python -u scripts/bench_lda.py --docs 125000 --strategy push_pull --local-server off --iters 5 > gpurun_out/r4b7/lda_share8_v$v.log 2>&1 || exit $?
done
timeout -k 10 300 python -u scripts/bench_lda.py --strategy push_pull --iters 5 > gpurun_out/r4b7/lda_full_local.log 2>&1
echo "rc=$?"
