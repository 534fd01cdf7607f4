set -o pipefail
O=gpurun_out/sc3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for k in 3 5 7; do
  timeout -k 10 300 python scripts/bench_subgraph.py --k $k > $O/k$k.log 2>&1 || exit 1
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o k7 -- python scripts/bench_subgraph.py --k 7 --iters 1 > $O/prof.log 2>&1 || exit 1
