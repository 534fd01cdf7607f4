#!/bin/bash
# LDA at K = 10,000 (BASELINE #5's published topic count): sparse sampler, full size, push-pull and rotation
set -o pipefail
O=gpurun_out/round5_w
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/bench_lda.py --docs 1000000 --topics 10000 --strategy push_pull --local-server off --iters 5 > $O/k10k_pp.log 2>&1 || { echo pp failed; tail $O/k10k_pp.log; exit 1; }
tail -1 $O/k10k_pp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('k10k pp', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'], d.get('pull_ms'), d.get('push_ms'))"
timeout -k 10 400 python -u scripts/bench_lda.py --docs 1000000 --topics 10000 --iters 5 > $O/k10k_rot.log 2>&1 || { echo rot failed; tail $O/k10k_rot.log; exit 1; }
tail -1 $O/k10k_rot.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('k10k rot', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
