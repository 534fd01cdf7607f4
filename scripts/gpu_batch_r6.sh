# Round-6 GPU validation batch: the whole GPU suite, then the bench (one JSON line).
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash scripts/gpu_batch_r6.sh <outdir>'
set -o pipefail
out=${1:-gpurun_out/r6_validate}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
timeout -k 10 300 python bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -5 "$out/bench.err"; exit 1; }
python -c "import json; r=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print(r['value'], r['sgd']['s_per_epoch'], r['pca']['eig_s'], r['pca']['s_per_pass'], r['lda']['tokens_per_sec'])"
