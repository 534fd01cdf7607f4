set -o pipefail
O=gpurun_out/sgdocc
mkdir -p $O
for v in 0 2 3 4; do
  timeout -k 10 240 python scripts/bench_sgd.py --epochs 3 --variant $v > $O/v$v.log 2>&1 || exit 1
done
