set -o pipefail
O=gpurun_out/${ALS_OUT:-als}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_als_gpu.py tests/test_apps_gpu.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -u scripts/bench_als.py > $O/bench_als.log 2>&1 || { tail -20 $O/bench_als.log; exit 1; }
tail -1 $O/bench_als.log
timeout -k 10 200 python -u scripts/bench_als.py --implicit 0 --factors 32 > $O/bench_als_exp32.log 2>&1 || exit 1
tail -1 $O/bench_als_exp32.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/bench_als.py --native-only > $O/prof.log 2>&1 || exit 1
