set -o pipefail
mkdir -p gpurun_out/sgd_xcd
O=gpurun_out/sgd_xcd
timeout -k 10 300 python -u -m pytest tests/test_sgd_mf_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 240 python scripts/bench_sgd.py --layout flat --epochs 3 > $O/flat.log 2>&1 || exit 1
for cfg in "64 256" "32 256" "128 256" "64 128" "32 512"; do
  set -- $cfg
  timeout -k 10 240 python scripts/bench_sgd.py --layout xcd --chunk $1 --blocks-per-xcd $2 --epochs 3 > $O/xcd_c$1_b$2.log 2>&1 || exit 1
done
