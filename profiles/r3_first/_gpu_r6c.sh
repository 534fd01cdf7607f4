#!/bin/bash
# round-3: new-kernel GPU tests (rowcodec, SGD flow, SVM, GMM), SGD flow A/B at the 8-GPU
# share and full size, full GPU suite, default bench, LDA push-pull sparse vs dense
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
timeout -k 10 400 python -u -m pytest tests/test_svm_gpu.py tests/test_gmm_gpu.py tests/test_rowcodec_gpu.py tests/test_sgd_flow_gpu.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r6c/pytest_new.log 2>&1
rc=$?; echo "new pytest rc=$rc"; grep -E "PASS|FAIL|x$|ms|device" gpurun_out/r6c/pytest_new.log | tail -30
case $rc in 0|1) ;; *) exit $rc;; esac
for v in 0 1; do
  timeout -k 10 200 python scripts/bench_sgd.py --ratings 12560063 --slices 16 --epochs 10 --variant $v --chunk 0 > gpurun_out/r6c/sgd_share_v$v.log 2>&1 || { echo "sgd share v$v failed"; tail -5 gpurun_out/r6c/sgd_share_v$v.log; exit 1; }
  echo "sgd 8-share v$v: $(grep '^{' gpurun_out/r6c/sgd_share_v$v.log | cut -c1-260)"
  timeout -k 10 200 python scripts/bench_sgd.py --epochs 5 --variant $v --chunk 0 > gpurun_out/r6c/sgd_full_v$v.log 2>&1 || { echo "sgd full v$v failed"; tail -5 gpurun_out/r6c/sgd_full_v$v.log; exit 1; }
  echo "sgd full v$v: $(grep '^{' gpurun_out/r6c/sgd_full_v$v.log | cut -c1-260)"
done
for m in "on --local-server off" "off --local-server off"; do
  timeout -k 10 240 python scripts/bench_lda.py --strategy push_pull --iters 5 --sparse-comm $m > gpurun_out/r6c/lda_pp.log 2>&1 || { echo "lda $m failed"; tail -5 gpurun_out/r6c/lda_pp.log; exit 1; }
  echo "lda $m: $(grep '^{' gpurun_out/r6c/lda_pp.log)"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6c/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r6c/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/r6c/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r6c/bench.log | cut -c1-600
