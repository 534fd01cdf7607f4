#!/bin/bash
# flow-kernel XCC map check + deterministic LDA layouts + de-flaked speed tests
mkdir -p gpurun_out/r5b
timeout -k 10 400 python -u -m pytest tests/test_sgd_flow_gpu.py tests/test_rowcodec_gpu.py tests/test_svm_gpu.py tests/test_gmm_gpu.py tests/test_eig_gpu.py tests/test_lda_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5b/pytest.log 2>&1
echo "pytest rc=$?"
