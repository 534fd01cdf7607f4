set -o pipefail
mkdir -p gpurun_out
for v in 0 1; do
  for sp in 0 103; do
    timeout -k 10 600 python scripts/bench_pca.py --steps 2 --variant $v --splits $sp > gpurun_out/bench_pca_v${v}_s${sp}.log 2>&1 || exit 1
  done
done
