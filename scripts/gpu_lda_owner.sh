# LDA owner slots (parallel/sparse_ps.py use_owner_slots): codec GPU tests, then push-pull
# sweeps with owner slots on / off at full size (K = 1000, 10000) and at the 8-rank share.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash scripts/gpu_lda_owner.sh [outdir]'
set -o pipefail
out=${1:-gpurun_out/r6_owner}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rowcodec_gpu.py -m gpu > $out/pytest_rowcodec.log 2>&1 || { tail -30 $out/pytest_rowcodec.log; exit 1; }
tail -1 $out/pytest_rowcodec.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python -u scripts/bench_lda.py --strategy push_pull --local-server off "$@" > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }
  python -c "import json,sys; r=json.loads(open('$out/$name.log').read().strip().splitlines()[-1]); print('$name', round(r['s_per_iter']*1e3,3), 'ms', r.get('pull_ms'), r.get('push_ms'))"
}
for o in on off; do run share8_$o --docs 125000 --topics 1000 --iters 10 --owner-slots $o; done
for o in on off; do run k1000_$o --topics 1000 --iters 5 --owner-slots $o; done
for o in on off; do run k10k_$o --topics 10000 --iters 3 --owner-slots $o; done
