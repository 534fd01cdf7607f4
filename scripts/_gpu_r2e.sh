#!/bin/bash
# round-2 app benches: LDA rotation + push-pull (packed plans), CCD allgather + rotation, PCA, TSQR
set -o pipefail
mkdir -p gpurun_out/r2e
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/r2e/$name.log 2>&1 || { tail -20 gpurun_out/r2e/$name.log; exit 1; }; tail -1 gpurun_out/r2e/$name.log | cut -c1-300; }
run lda_rot python scripts/bench_lda.py --strategy rotation
run lda_pp python scripts/bench_lda.py --strategy push_pull
run ccd_ag python scripts/bench_ccd.py --mode allgather
run ccd_rot python scripts/bench_ccd.py --mode rotation
run pca python scripts/bench_pca.py --steps 2
run tsqr python scripts/bench_tsqr.py
run syrk_diag python scripts/syrk_diag.py
run syrk_diag_s24 python scripts/syrk_diag.py --splits 24
