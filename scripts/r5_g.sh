#!/bin/bash
# fused sparse-sampler rows with wave-aggregated push-slot reservations vs unfused, full size
set -o pipefail
O=gpurun_out/round5_g
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lda_pp_mp_gpu.py tests/test_rowcodec_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for F in on off; do
  timeout -k 10 300 python -u scripts/bench_lda.py --docs 1e6 --strategy push_pull --local-server off --iters 5 --fused-rows $F > $O/full_$F.log 2>&1 || { echo full failed; tail $O/full_$F.log; exit 1; }
  tail -1 $O/full_$F.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused', '$F', d['s_per_iter'], d['value'], d['loglik_end'], d.get('pull_ms'), d.get('push_ms'))"
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 2 --warmup 1 --points 1e7 --sgd off --pca-n 1e6 --pca-steps 2 > $O/bench_lda.json 2> $O/bench_lda.err || { echo bench failed; tail $O/bench_lda.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_lda.json'))['lda']; print({k: d[k] for k in ('tokens_per_sec','s_per_iter','comm_mode','fused_rows','sampler')}, d.get('local_server_alias'))"
