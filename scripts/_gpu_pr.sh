set -o pipefail
O=gpurun_out/pr
mkdir -p $O
export TMPDIR=/tmp
true
timeout -k 10 150 python -u scripts/bench_pagerank.py > $O/bench_pagerank.log 2>&1 || { tail -20 $O/bench_pagerank.log; exit 1; }
timeout -k 10 150 python -u scripts/bench_pagerank.py --degree 4 > $O/bench_pagerank_d4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/bench_pagerank.py --iters 10 > $O/prof.log 2>&1 || exit 1
tail -1 $O/bench_pagerank.log; tail -1 $O/bench_pagerank_d4.log
