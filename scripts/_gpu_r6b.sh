#!/bin/bash
# round-3: rowcodec + LDA sparse rows, MF-SGD flow kernel (GPU tests + 8-GPU-share A/B),
# full GPU suite, default bench, LDA push-pull sparse vs dense at 1M x 1M x 1000
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6b
timeout -k 10 300 python -u -m pytest tests/test_rowcodec_gpu.py tests/test_sgd_flow_gpu.py tests/test_svm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b/pytest_new.log 2>&1
rc=$?; echo "new pytest rc=$rc"; tail -5 gpurun_out/r6b/pytest_new.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  timeout -k 10 200 python scripts/bench_sgd.py --ratings 12560063 --slices 16 --epochs 10 --variant $v --chunk 0 > gpurun_out/r6b/sgd_share_v$v.log 2>&1 || { echo "sgd share v$v failed"; tail -5 gpurun_out/r6b/sgd_share_v$v.log; exit 1; }
  echo "sgd 8-share v$v: $(grep '^{' gpurun_out/r6b/sgd_share_v$v.log | cut -c1-300)"
  timeout -k 10 200 python scripts/bench_sgd.py --epochs 5 --variant $v > gpurun_out/r6b/sgd_full_v$v.log 2>&1 || { echo "sgd full v$v failed"; tail -5 gpurun_out/r6b/sgd_full_v$v.log; exit 1; }
  echo "sgd full v$v: $(grep '^{' gpurun_out/r6b/sgd_full_v$v.log | cut -c1-300)"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6b/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r6b/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/r6b/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r6b/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
for m in "on --local-server off" "off --local-server off"; do
  timeout -k 10 240 python scripts/bench_lda.py --strategy push_pull --iters 5 --sparse-comm $m > gpurun_out/r6b/lda_pp.log 2>&1 || { echo "lda $m failed"; tail -5 gpurun_out/r6b/lda_pp.log; exit 1; }
  echo "lda $m: $(grep '^{' gpurun_out/r6b/lda_pp.log)"
done
