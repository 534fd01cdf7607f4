#!/bin/bash
# LDA A/B with run-to-run repeats: baseline (LDS topic deltas) vs + per-wave word-row deltas
set -o pipefail
mkdir -p gpurun_out/r3d
for rep in 1 2 3; do
  for lib in base new; do
    if [ $lib = base ]; then export HARP_KERNEL_LIB=$PWD/alt_libs/libharp_kernels_base.so; else unset HARP_KERNEL_LIB; fi
    timeout -k 10 300 python scripts/bench_lda.py --iters 5 > gpurun_out/r3d/${lib}_$rep.log 2>&1 || { tail -5 gpurun_out/r3d/${lib}_$rep.log; exit 1; }
    python -c "import json; r=json.loads(open('gpurun_out/r3d/${lib}_$rep.log').read().strip().splitlines()[-1]); print('$lib', $rep, round(r['s_per_iter'],5), r['loglik_end'])"
  done
done
