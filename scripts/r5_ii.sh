#!/bin/bash
# LDA rotation (collective mapper) at full size after the round-5 sampler changes: K = 1000 (dense default) and K = 10,000 (sparse)
set -o pipefail
O=gpurun_out/round5_ii
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --iters 5 > $O/rot_k1k.log 2>&1 || { echo rot failed; tail $O/rot_k1k.log; exit 1; }
tail -1 $O/rot_k1k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rot k1k', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --strategy push_pull --iters 5 > $O/pp_local_k1k.log 2>&1 || { echo pp failed; tail $O/pp_local_k1k.log; exit 1; }
tail -1 $O/pp_local_k1k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pp local k1k', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
