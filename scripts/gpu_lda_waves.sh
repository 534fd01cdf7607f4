# Sparse LDA sampler workgroup size at K = 10,000 (HARP_LDA_SPARSE_WAVES: 8 = six waves per
# SIMD at 74 VGPRs, 16 = eight per SIMD at 64 VGPRs): rotation and push-pull sweeps.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash scripts/gpu_lda_waves.sh [outdir]'
set -o pipefail
out=${1:-gpurun_out/r6_waves}
mkdir -p $out
run() {  # name, waves, args...
  local name=$1 w=$2; shift 2
  HARP_LDA_SPARSE_WAVES=$w timeout -k 10 400 python -u scripts/bench_lda.py "$@" > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }
  python -c "import json,sys; r=json.loads(open('$out/$name.log').read().strip().splitlines()[-1]); print('$name', round(r['s_per_iter']*1e3,3), 'ms', r.get('loglik_end'))"
}
for w in 16 8; do
  run rot_w$w $w --topics 10000 --strategy rotation --iters 3
  run pp_w$w $w --topics 10000 --strategy push_pull --local-server off --iters 3
done
