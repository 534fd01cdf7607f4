set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ccd_gpu.py -x -q > gpurun_out/ccd_gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 python scripts/bench_ccd.py --iters 3 > gpurun_out/bench_ccd.log 2>&1
