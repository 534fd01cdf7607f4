#!/bin/bash
# round-3: MF-SGD with hot-row weighted item blocks as the default: GPU tests + bench record
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r9f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_sgd_mf_gpu.py tests/test_sgd_flow_gpu.py -q --timeout 200 --timeout-method thread > $O/pytest_sgd.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_sgd.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --extras off > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"
grep '^{' $O/bench.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); s=r["sgd"]; print(r["value"], s["updates_per_sec"], s["median_updates_per_sec"], s["s_per_epoch"], s["train_rmse"])'
exit $rc
