#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r7j
mkdir -p $O
timeout -k 10 200 python scripts/probe_eig_nb.py > $O/nb.log 2>&1 || { tail -5 $O/nb.log; exit 1; }
grep '^{' $O/nb.log
cd /tmp && HARP_EIG_NB=32 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof7j -o run -- python $GRAFT_REPO_ROOT/scripts/probe_eig_nb.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find /tmp/prof7j -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
python3 - <<'PY'
import csv, os
rows = list(csv.DictReader(open(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r7j/kernel_stats.csv")))
for r in rows[:8]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
