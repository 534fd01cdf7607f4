set -o pipefail
O=gpurun_out/sgd_wide
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_sgd_mf_gpu.py -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_sgd.py --epochs 2 --rank 2000 > $O/r2000_c64.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_sgd.py --epochs 2 --rank 2000 --chunk 128 --blocks-per-xcd 64 > $O/r2000_c128_b64.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_sgd.py --epochs 2 --rank 512 > $O/r512.log 2>&1 || exit 1
