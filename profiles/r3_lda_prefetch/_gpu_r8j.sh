#!/bin/bash
# round-3: LDA doc-list prefetch -- likelihood after 20 sweeps, base vs new (push-pull), 2 runs each
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r8j
mkdir -p $O
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export HARP_KERNEL_LIB=$GRAFT_REPO_ROOT/abtest/libharp_kernels_base.so; else unset HARP_KERNEL_LIB; fi
    timeout -k 10 200 python scripts/bench_lda.py --iters 20 --strategy push_pull --seed $rep > $O/${v}_$rep.log 2>&1 || timeout -k 10 200 python scripts/bench_lda.py --iters 20 --strategy push_pull > $O/${v}_$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/${v}_$rep.log; exit 1; }
    echo "$v rep$rep: $(grep '^{' $O/${v}_$rep.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["loglik_init"], r["loglik_end"], round(r["s_per_iter"],5))')"
  done
done
