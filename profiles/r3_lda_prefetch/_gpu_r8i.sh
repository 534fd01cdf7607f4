#!/bin/bash
# round-3: LDA sparse sampler with the next token's doc list prefetched (A/B against the
# previous kernel library, alternating), plus the LDA GPU tests on the new kernel
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lda_gpu.py -q --timeout 200 --timeout-method thread > $O/pytest_lda.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_lda.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export HARP_KERNEL_LIB=$GRAFT_REPO_ROOT/abtest/libharp_kernels_base.so; else unset HARP_KERNEL_LIB; fi
    for st in push_pull rotation; do
      timeout -k 10 200 python scripts/bench_lda.py --iters 5 --strategy $st > $O/${v}_${st}_$rep.log 2>&1 || { echo "$v $st failed"; tail -5 $O/${v}_${st}_$rep.log; exit 1; }
      echo "$v $st rep$rep: $(grep '^{' $O/${v}_${st}_$rep.log | cut -c1-260)"
    done
  done
done
