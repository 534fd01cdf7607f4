#!/bin/bash
# round-3 first GPU check: GPU tests (tuner, rowcodec, bench records), default bench with
# every nested record, LDA push-pull sparse rows vs dense at 1M x 1M x 1000 on one GPU
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6a
timeout -k 10 300 python -u -m pytest tests/test_rowcodec_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6a/pytest_rowcodec.log 2>&1
rc=$?; echo "rowcodec pytest rc=$rc"; tail -5 gpurun_out/r6a/pytest_rowcodec.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6a/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r6a/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/r6a/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r6a/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
for m in "on --local-server off" "off --local-server off" "auto"; do
  timeout -k 10 240 python scripts/bench_lda.py --strategy push_pull --iters 5 --sparse-comm $m > gpurun_out/r6a/lda_pp.log 2>&1 || { echo "lda $m failed"; tail -5 gpurun_out/r6a/lda_pp.log; exit 1; }
  echo "lda $m: $(grep '^{' gpurun_out/r6a/lda_pp.log)"
done
