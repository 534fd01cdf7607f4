set -o pipefail
O=gpurun_out/mlr3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mlr_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for t in 256 512 1024; do
HARP_MLR_THREADS=$t timeout -k 10 300 python scripts/bench_mlr.py --alpha 0.05 > $O/bench_t$t.log 2>&1 || exit 1
HARP_MLR_THREADS=$t timeout -k 10 300 python scripts/bench_mlr.py --batch 1 --rows 4000 > $O/bench_b1_t$t.log 2>&1 || exit 1
done
HARP_MLR_THREADS=1024 timeout -k 10 300 python -u -m pytest tests/test_mlr_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_1024.log 2>&1 || exit 1
