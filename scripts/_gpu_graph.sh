set -o pipefail
O=gpurun_out/sgdwin
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sgd_mf_gpu.py -x -v --timeout 120 --timeout-method thread > $O/test.log 2>&1 || exit 1
timeout -k 10 240 python scripts/bench_sgd.py --epochs 3 > $O/bench_sgd.log 2>&1 || exit 1
