set -o pipefail
O=gpurun_out/sgd_xcd8
mkdir -p $O
for v in 0 1; do
  timeout -k 10 240 python scripts/bench_sgd.py --layout xcd --chunk 64 --blocks-per-xcd 128 --variant $v --epochs 3 > $O/v$v.log 2>&1 || exit 1
done
