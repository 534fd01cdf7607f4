#!/bin/bash
# round-5 validation (output dir as the argument): full GPU suite, smoke, default bench, kernel stats of the bench
set -o pipefail
O=gpurun_out/${1:-round5_v3}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
O=$O python - <<'PY'
import json, os
d = json.loads(open(os.environ["O"] + "/bench.json").read().strip().splitlines()[-1])
print("kmeans", d["value"], d["unit"])
for k in ("sgd", "pca", "lda"):
    r = d.get(k, {})
    print(k, {x: r.get(x) for x in ("updates_per_sec", "s_per_epoch", "s_per_pass", "eig_s", "tokens_per_sec", "s_per_iter", "sampler") if x in r})
PY
