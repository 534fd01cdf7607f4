#!/bin/bash
# round-3: LDA sparse sampler -- deeper load pipeline (ids two tokens ahead, doc range one
# ahead) vs the one-token doc-list prefetch (base library), and workgroup size, push-pull
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lda_gpu.py -q --timeout 200 --timeout-method thread > $O/pytest_lda.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_lda.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base new new16; do
    unset HARP_KERNEL_LIB HARP_LDA_SPARSE_WAVES
    [ $v = base ] && export HARP_KERNEL_LIB=$GRAFT_REPO_ROOT/abtest/libharp_kernels_base.so
    [ $v = new16 ] && export HARP_LDA_SPARSE_WAVES=16
    timeout -k 10 200 python scripts/bench_lda.py --iters 5 --strategy push_pull > $O/${v}_$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/${v}_$rep.log; exit 1; }
    echo "$v rep$rep: $(grep '^{' $O/${v}_$rep.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_iter"],5), r["loglik_end"])')"
  done
done
