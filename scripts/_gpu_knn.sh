set -o pipefail
O=gpurun_out/knn2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_knn.py > $O/bench_knn.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_knn.py --k 4 --dim 32 > $O/bench_knn_k4.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o knn -- python3 $GRAFT_REPO_ROOT/scripts/bench_knn.py --reps 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
