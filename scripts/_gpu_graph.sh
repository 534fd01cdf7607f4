set -o pipefail
O=gpurun_out/ldapf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lda_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_v0.log 2>&1 || exit 1
HARP_LDA_VARIANT=1 timeout -k 10 300 python -u -m pytest tests/test_lda_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_v1.log 2>&1 || exit 1
timeout -k 10 400 python scripts/bench_lda.py --iters 3 > $O/bench_v0.log 2>&1 || exit 1
HARP_LDA_VARIANT=1 timeout -k 10 400 python scripts/bench_lda.py --iters 3 > $O/bench_v1.log 2>&1 || exit 1
