set -o pipefail
O=gpurun_out/kcsr
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kmeans_csr_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_kmeans_csr.py > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_kmeans_csr.py --centroids 1000 --rows 200000 > $O/bench_k1000.log 2>&1 || exit 1
