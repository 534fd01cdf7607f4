set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_lda_gpu.py -x -q > gpurun_out/lda_gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 python scripts/bench_lda.py --strategy rotation --iters 3 > gpurun_out/bench_lda_rot16.log 2>&1 || exit 1
timeout -k 10 900 python scripts/bench_lda.py --strategy push_pull --iters 3 > gpurun_out/bench_lda_pp16.log 2>&1
