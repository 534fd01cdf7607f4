#!/bin/bash
# bench.py with the nested PCA / LDA records (default N=1 run, as the driver runs it)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a
s=$(date +%s)
timeout -k 10 600 python bench.py > gpurun_out/r5a/bench.log 2>&1 || { tail -30 gpurun_out/r5a/bench.log; exit 1; }
echo "wall $(( $(date +%s) - s )) s"
grep '^{' gpurun_out/r5a/bench.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value']); print(r['sgd']); print(r['pca']); print(r['lda'])"
