set -o pipefail
O=gpurun_out/sgdlayout
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sgd_mf_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || exit 1
for v in 0 2; do
  timeout -k 10 240 python scripts/bench_sgd.py --epochs 3 --variant $v > $O/v$v.log 2>&1 || exit 1
done
timeout -k 10 240 python scripts/bench_sgd.py --epochs 3 --layout flat > $O/flat.log 2>&1 || exit 1
timeout -k 10 240 python scripts/bench_sgd.py --epochs 3 --skew 1 > $O/skew1.log 2>&1 || exit 1
