set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests2.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_v14.log 2>&1
