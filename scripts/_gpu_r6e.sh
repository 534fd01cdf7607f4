#!/bin/bash
# round-3: SMO v3 (512-thread form, batched gathers), MF-SGD flow vs per-sub-step kernel
# traces at the 8-GPU share, SYRK bottleneck split (no lock-step hint)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_svm_gpu.py -v -s --timeout 250 --timeout-method thread > $O/pytest_svm.log 2>&1
rc=$?; echo "svm pytest rc=$rc"; grep -E "PASS|FAIL|device " $O/pytest_svm.log | tail -12
case $rc in 0|1) ;; *) exit $rc;; esac
cd /tmp
for v in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_v$v -o run -- python3 $R/scripts/bench_sgd.py --ratings 12560063 --slices 16 --epochs 3 --variant $v --chunk 0 > $O/prof_v$v.log 2>&1 || { echo "prof v$v failed"; tail -5 $O/prof_v$v.log; exit 1; }
  f=$(find /tmp/prof_v$v -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_v$v.csv; head -5 $f | cut -c1-220
done
cd $R
timeout -k 10 300 python scripts/syrk_diag.py --modes 0,1,3,5,6 > $O/syrk_diag.log 2>&1 || { echo "syrk diag failed"; tail -5 $O/syrk_diag.log; exit 1; }
tail -3 $O/syrk_diag.log
