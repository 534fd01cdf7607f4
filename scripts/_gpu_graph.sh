set -o pipefail
O=gpurun_out/hostfix
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kmeans_gpu.py tests/test_apps_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || exit 1
for pts in 1e6 1.25e7 2.5e7; do
  timeout -k 10 200 python bench.py --points $pts --steps 20 --warmup 3 > $O/b_$pts.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --points $pts --steps 20 --warmup 3 --graph > $O/g_$pts.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/full.log 2>&1 || exit 1
