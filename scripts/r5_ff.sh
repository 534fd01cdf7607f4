#!/bin/bash
# encode-once pull: rowcodec + multi-rank LDA GPU tests, then the P=2 / P=4 one-GPU rehearsal of the LDA record
set -o pipefail
O=gpurun_out/round5_ff
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp HARP_BENCH_TRACE=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rowcodec_gpu.py tests/test_lda_pp_mp_gpu.py tests/test_lda_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for P in 2 4; do
  timeout -k 10 400 python bench.py --gpus $P --backend gloo --steps 2 --warmup 1 --points 2e6 --sgd off --extras on --pca-n 1e6 --pca-steps 2 --lda-docs 4e5 --lda-vocab 4e5 --lda-iters 3 --extras-timeout 300 > $O/bench_p$P.log 2>&1 || { echo "bench P=$P failed"; tail -20 $O/bench_p$P.log; exit 1; }
  grep '^{' $O/bench_p$P.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); v=r.get("lda",{}); print("P", r["n_gpus"], {a:b for a,b in v.items() if a in ("tokens_per_sec","s_per_iter","comm_mode","fused_rows","error","loglik_end","pull_ms","push_ms")})'
done
