#!/bin/bash
# round-3: SGD flow kernel v2 (per-block completion) A/B + kernel traces, SVM speed,
# LDA tuner GPU test, then the rest of the GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6d
timeout -k 10 300 python -u -m pytest tests/test_svm_gpu.py tests/test_sgd_flow_gpu.py tests/test_lda_gpu.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r6d/pytest_new.log 2>&1
rc=$?; echo "new pytest rc=$rc"; grep -E "PASS|FAIL|x$|device " gpurun_out/r6d/pytest_new.log | tail -30
case $rc in 0|1) ;; *) exit $rc;; esac
for v in 0 1; do
  timeout -k 10 200 python scripts/bench_sgd.py --ratings 12560063 --slices 16 --epochs 10 --variant $v --chunk 0 > gpurun_out/r6d/sgd_share_v$v.log 2>&1 || { echo "sgd share v$v failed"; tail -5 gpurun_out/r6d/sgd_share_v$v.log; exit 1; }
  echo "sgd 8-share v$v: $(grep '^{' gpurun_out/r6d/sgd_share_v$v.log | cut -c100-260)"
done
cd /tmp
for v in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6d/prof_v$v -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_sgd.py --ratings 12560063 --slices 16 --epochs 3 --variant $v --chunk 0 > $GRAFT_REPO_ROOT/gpurun_out/r6d/prof_v$v.log 2>&1 || { echo "prof v$v failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/r6d/prof_v$v.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
find gpurun_out/r6d -name "*kernel_stats.csv" | head
for f in $(find gpurun_out/r6d -name "*kernel_stats.csv"); do echo $f; head -6 $f | cut -c1-200; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6d/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r6d/pytest_gpu.log
