#!/bin/bash
# chunked side-stream bucket pipeline: numerics test, then the 1-GPU bench per chunk count
set -o pipefail
mkdir -p gpurun_out/r2h
timeout -k 10 300 python -u -m pytest tests/test_kmeans_gpu.py -x -q --timeout 120 --timeout-method thread -k "chunked or bucket" > gpurun_out/r2h/pytest.log 2>&1 || { tail -40 gpurun_out/r2h/pytest.log; exit 1; }
tail -2 gpurun_out/r2h/pytest.log
for c in 1 2 4 8 1; do
  HARP_KMEANS_CHUNKS=$c timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sgd off > gpurun_out/r2h/bench_c$c.log 2>&1 || { tail -20 gpurun_out/r2h/bench_c$c.log; exit 1; }
  echo "chunks=$c $(tail -1 gpurun_out/r2h/bench_c$c.log | cut -c1-120)"
done
cd /tmp && export TMPDIR=/tmp && HARP_KMEANS_CHUNKS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2h/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --sgd off > $GRAFT_REPO_ROOT/gpurun_out/r2h/prof.log 2>&1
echo prof rc=$?
