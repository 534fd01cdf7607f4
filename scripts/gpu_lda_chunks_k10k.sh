# Sparse LDA sampler chunk size at K = 10,000 (rotation and push-pull, full size): the
# LDAConfig default (65536 tokens at this size) against smaller chunks.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash scripts/gpu_lda_chunks_k10k.sh [outdir]'
set -o pipefail
out=${1:-gpurun_out/r6_chunks}
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 300 python -u scripts/bench_lda.py --topics 10000 --iters 3 "$@" > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }
  python -c "import json,sys; r=json.loads(open('$out/$name.log').read().strip().splitlines()[-1]); print('$name', round(r['s_per_iter']*1e3,3), 'ms', r.get('max_chunk'), r.get('loglik_end'))"
}
for mc in 4096 16384; do run rot_mc$mc --strategy rotation --max-chunk $mc; done
run rot_default --strategy rotation
for mc in 4096 16384; do run pp_mc$mc --strategy push_pull --local-server off --max-chunk $mc; done
