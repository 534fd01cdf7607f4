set -o pipefail
O=gpurun_out/lda_sparse6
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lda_gpu.py -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
B="timeout -k 10 300 python scripts/bench_lda.py --iters 3"
$B --topics 10000 > $O/k10000_w8.log 2>&1 || exit 1
$B > $O/k1000_dense.log 2>&1 || exit 1
HARP_LDA_SAMPLER=sparse $B > $O/k1000_sparse_w8.log 2>&1 || exit 1
HARP_LDA_SAMPLER=sparse HARP_LDA_SPARSE_WAVES=4 $B > $O/k1000_sparse_w4.log 2>&1 || exit 1
