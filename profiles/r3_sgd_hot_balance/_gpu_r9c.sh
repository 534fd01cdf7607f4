#!/bin/bash
# round-3: MF-SGD one slice per rank, item-popularity skew 1 (uniform) vs 2 (default), and the
# kernel trace of the skewed epoch (per-launch spread)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r9c
mkdir -p $O
for sk in 1.0 2.0 3.0; do
  timeout -k 10 200 python scripts/bench_sgd.py --epochs 10 --skew $sk > $O/skew$sk.log 2>&1 || exit 1
  echo "skew $sk: $(grep '^{' $O/skew$sk.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["s_per_epoch"]*1e3,3), "ms", r["value"])')"
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/p9c -o run -- python $GRAFT_REPO_ROOT/scripts/bench_sgd.py --epochs 3 > $O/prof.log 2>&1
find /tmp/p9c -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
python3 - <<'PY'
import csv, os
rows = list(csv.DictReader(open(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r9c/kernel_trace.csv")))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "mf_sgd_xcd" in r["Kernel_Name"]]
print("mf_sgd_xcd launches", len(d), "us:", [round(x) for x in d[-16:]])
PY
