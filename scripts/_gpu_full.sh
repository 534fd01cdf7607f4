set -o pipefail
O=gpurun_out/${FULL_OUT:-full5}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || exit 1
timeout -k 10 240 python scripts/bench_sgd.py --epochs 5 > $O/bench_sgd.log 2>&1 || exit 1
timeout -k 10 400 python scripts/bench_lda.py --iters 3 > $O/bench_lda.log 2>&1 || exit 1
timeout -k 10 400 python scripts/bench_lda.py --iters 3 --strategy push_pull > $O/bench_lda_pp.log 2>&1 || exit 1
timeout -k 10 400 python scripts/bench_lda.py --iters 3 --topics 10000 > $O/bench_lda_k10k.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_pca.py > $O/bench_pca.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_ccd.py > $O/bench_ccd.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_subgraph.py > $O/bench_subgraph.log 2>&1 || exit 1
