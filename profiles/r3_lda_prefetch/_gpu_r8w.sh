#!/bin/bash
# round-3: LDA sparse sampler with one barrier per chunk start (A/B vs the previous library),
# full corpus and the 8-GPU share (docs / 8, full vocabulary), push-pull
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8w
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lda_gpu.py -q --timeout 200 --timeout-method thread > $O/pytest_lda.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_lda.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base new; do
    unset HARP_KERNEL_LIB
    [ $v = base ] && export HARP_KERNEL_LIB=$GRAFT_REPO_ROOT/abtest/libharp_kernels_base.so
    for docs in 1000000 125000; do
      timeout -k 10 200 python scripts/bench_lda.py --iters 5 --strategy push_pull --docs $docs > $O/${v}_d${docs}_$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/${v}_d${docs}_$rep.log; exit 1; }
      echo "$v docs=$docs rep$rep: $(grep '^{' $O/${v}_d${docs}_$rep.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_iter"],5), r["loglik_end"])')"
    done
  done
done
