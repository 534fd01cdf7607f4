#!/bin/bash
# LDA with auto word slices (1 on one worker): GPU tests + rotation at full size
set -o pipefail
O=gpurun_out/round5_kk
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lda_gpu.py tests/test_rowcodec_gpu.py tests/test_lda_pp_mp_gpu.py tests/test_slabcodec_gpu.py \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/bench_lda.py --docs 1000000 --iters 5 > $O/rot_auto.log 2>&1 || { echo rot failed; tail $O/rot_auto.log; exit 1; }
tail -1 $O/rot_auto.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rot auto', d['s_per_iter'], d['value'], d['loglik_end'], d['sampler'])"
