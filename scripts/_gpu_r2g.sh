#!/bin/bash
# LDA push-pull: dense vs sparse push/pull cost on 1 GPU (K=1000 and K=10,000)
set -o pipefail
mkdir -p gpurun_out/r2g
for cfg in "1000 off" "1000 on" "10000 off" "10000 on"; do set -- $cfg
  timeout -k 10 300 python scripts/bench_lda.py --strategy push_pull --topics $1 --sparse-comm $2 > gpurun_out/r2g/pp_k$1_$2.log 2>&1 || { tail -20 gpurun_out/r2g/pp_k$1_$2.log; exit 1; }
  echo "K$1 sparse=$2 $(grep -o '"s_per_iter": [0-9.e-]*' gpurun_out/r2g/pp_k$1_$2.log)"
done
