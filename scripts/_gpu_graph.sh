set -o pipefail
O=gpurun_out/ldamap
mkdir -p $O
for v in 0 1 3; do
  HARP_LDA_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_lda_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_v$v.log 2>&1 || exit 1
done
for v in 0 2 3 4; do
  HARP_LDA_VARIANT=$v timeout -k 10 400 python scripts/bench_lda.py --iters 3 > $O/bench_v$v.log 2>&1 || exit 1
done
