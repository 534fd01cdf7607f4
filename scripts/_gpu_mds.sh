set -o pipefail
O=gpurun_out/mds
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mds_gpu.py tests/test_mlr_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_mds.py > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_mlr.py --batch 1 --rows 4000 > $O/bench_mlr_b1_auto.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_mlr.py --alpha 0.05 > $O/bench_mlr_auto.log 2>&1 || exit 1
