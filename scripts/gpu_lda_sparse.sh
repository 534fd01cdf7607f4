# LDA sparse sampler (K > 1024) checks and sweeps: GPU tests of the sparse / fused paths, then
# K = 10,000 push-pull (owner slots) and rotation sweeps at full size.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash scripts/gpu_lda_sparse.sh [outdir]'
set -o pipefail
out=${1:-gpurun_out/r6_sparse}
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lda_gpu.py tests/test_rowcodec_gpu.py -m gpu > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python -u scripts/bench_lda.py "$@" > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }
  python -c "import json,sys; r=json.loads(open('$out/$name.log').read().strip().splitlines()[-1]); print('$name', round(r['s_per_iter']*1e3,3), 'ms', r.get('pull_ms'), r.get('push_ms'), r.get('loglik_end'))"
}
run k10k_pp --topics 10000 --strategy push_pull --local-server off --iters 3
run k10k_rot --topics 10000 --strategy rotation --iters 3
